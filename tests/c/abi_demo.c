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
    /* the same 100 steps as 4 launches of the K-step rollout (random policy
       drawn in the kernel): the last step's obs and every ep_num bitwise */
    dr_handle *h2 = NULL;
    {
        dr_handle *hsave = h;
        h = NULL;
        CK(dr_create(&cfg, &h2));
        h = hsave;
    }
    const int K = 25;
    float *obs_k, *rew_k;
    uint8_t *done_k;
    if (hipMalloc((void **)&obs_k, (size_t)K * n * 60) ||
        hipMalloc((void **)&rew_k, (size_t)K * n * 4) || hipMalloc((void **)&done_k, (size_t)K * n))
        return 11;
    CK(dr_reset(h2, obs, s));
    for (int c = 0; c < 100 / K; ++c)
        CK(dr_rollout_random(h2, K, 7, (int64_t)c * K, 0.0f, 7.3575f, NULL, obs_k, rew_k,
                             done_k, s));
    CK(dr_get_state(h2, DR_FIELD_EP_NUM, ep, s));
    if (hipStreamSynchronize(s)) return 12;
    float *ho2 = malloc(n * 60);
    int32_t *he2 = malloc(n * 4);
    if (hipMemcpy(ho2, obs_k + (size_t)(K - 1) * n * 15, n * 60, hipMemcpyDeviceToHost) ||
        hipMemcpy(he2, ep, n * 4, hipMemcpyDeviceToHost))
        return 13;
    for (int64_t i = 0; i < n * 15; ++i)
        if (ho2[i] != ho[i] && !(isnan(ho2[i]) && isnan(ho[i]))) return 14;
    for (int64_t i = 0; i < n; ++i)
        if (he2[i] != he[i]) return 15;
    CK(dr_destroy(h2));
    CK(dr_destroy(h));
    printf("c abi ok: %ld episodes finished; dr_rollout_random == dr_step\n", episodes);
    return 0;
}
