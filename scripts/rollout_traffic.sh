#!/bin/bash
# HBM traffic of the headline rollout kernel (env_rollout_*, 65,536 envs,
# f64, actions from HBM) at K = 32 steps per launch (bench.py's default
# --steps 1000 form; 960 steps = 30 full launches here) and K = 20 (the
# driver's --steps 20 form), and of the bench line's companion_rollout
# (4,194,304 envs, K = 32, the one-role env_rollout_kernel), FETCH_SIZE and
# WRITE_SIZE in separate PMC passes
# (MI355X_MICROARCH.md: FETCH_SIZE x 2 on gfx950), written into
# profiles/traffic.json by scripts/traffic_update.py.
cd "$(dirname "$0")/.."
OUT=$PWD/gpurun_out/pmc_rollout_traffic
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 32 20; do
  if [ $k = 32 ]; then ARGS="--steps 960 --warmup 64"; else ARGS="--steps 20 --warmup 20"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/k${k}_$c" -o run \
        -- python3 "$PWD/bench.py" --no-cpu-baseline --no-companion --no-graph --ppo-updates 0 \
        --rollout-k 0 $ARGS > "$OUT/k${k}_$c.log" 2>&1
    rc=$?; echo "k=$k $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/k${k}_$c.log"; exit $rc; fi
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/c4m_$c" -o run \
      -- python3 "$PWD/bench.py" --no-cpu-baseline --no-graph --ppo-updates 0 --rollout-k 0 \
      --steps 20 --warmup 5 > "$OUT/c4m_$c.log" 2>&1
  rc=$?; echo "companion $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/c4m_$c.log"; exit $rc; fi
done
python3 scripts/traffic_update.py "$OUT"
