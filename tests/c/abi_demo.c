/* Plain-C consumer of the libdronerl C ABI (include/dronerl.h): what a
 * non-Python host binding does.  Build (see tests/test_c_abi.py):
 *   gcc -std=c11 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
 *       tests/c/abi_demo.c -Ldrone_rl_amd -ldronerl -L/opt/rocm/lib -lamdhip64
 * Steps 4096 envs x 100 random-policy steps and checks the outputs. */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "dronerl.h"

#define CK(x)                                                             \
    do {                                                                  \
        int rc__ = (x);                                                   \
        if (rc__ != 0) {                                                  \
            fprintf(stderr, "%s failed: %d (%s)\n", #x, rc__,             \
                    dr_last_error(h));                                    \
            return 1;                                                     \
        }                                                                 \
    } while (0)

int main(void) {
    const int64_t n = 4096;
    dr_handle *h = NULL;
    dr_config cfg = {0};
    cfg.num_envs = n;
    cfg.variant = DR_VARIANT_GYM;
    cfg.state_dtype = DR_STATE_F64;
    cfg.rng_mode = DR_RNG_PHILOX;
    cfg.auto_reset = 1;
    cfg.seed = 42;
    if (dr_abi_version() != DR_ABI_VERSION) return 2;
    CK(dr_create(&cfg, &h));
    float *act, *obs, *rew;
    uint8_t *done;
    int32_t *ep;
    if (hipMalloc((void **)&act, n * 16) || hipMalloc((void **)&obs, n * 60) ||
        hipMalloc((void **)&rew, n * 4) || hipMalloc((void **)&done, n) ||
        hipMalloc((void **)&ep, n * 4))
        return 3;
    hipStream_t s;
    if (hipStreamCreate(&s)) return 4;
    CK(dr_reset(h, obs, s));
    for (int t = 0; t < 100; ++t) {
        CK(dr_random_actions(n, 7, 0, t, 0.0f, 7.3575f, act, s));
        CK(dr_step(h, act, obs, rew, done, NULL, s));
    }
    CK(dr_get_state(h, DR_FIELD_EP_NUM, ep, s));
    if (hipStreamSynchronize(s)) return 5;
    float *hr = malloc(n * 4), *ho = malloc(n * 60);
    int32_t *he = malloc(n * 4);
    if (hipMemcpy(hr, rew, n * 4, hipMemcpyDeviceToHost) ||
        hipMemcpy(ho, obs, n * 60, hipMemcpyDeviceToHost) ||
        hipMemcpy(he, ep, n * 4, hipMemcpyDeviceToHost))
        return 6;
    long episodes = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!isfinite(hr[i]) || hr[i] > 1.0f || hr[i] < -5.0f) return 7;
        episodes += he[i] - 2;      /* ctor reset + dr_reset -> ep_num 2 */
    }
    for (int64_t i = 0; i < n * 15; ++i)
        if (!isfinite(ho[i])) return 8;
    if (episodes < n) return 9;     /* random policy: ~3 episodes / 100 steps */
    /* error path: a misaligned action pointer is rejected, not dereferenced */
    if (dr_step(h, act + 1, obs, rew, done, NULL, s) != DR_ERR_INVALID) return 10;
    CK(dr_destroy(h));
    printf("c abi ok: %ld episodes finished\n", episodes);
    return 0;
}
