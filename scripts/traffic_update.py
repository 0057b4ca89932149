"""Per-launch HBM bytes of the headline rollout kernel from the PMC passes of
scripts/rollout_traffic.sh, merged into profiles/traffic.json (read by
bench.py for the headline's roofline.traffic).

Bytes per launch = FETCH_SIZE x 2 (the gfx950 correction of
MI355X_MICROARCH.md) + WRITE_SIZE, both KiB -> B, averaged over the
env_rollout_kernel dispatches of each pass (the K-step launches only).
Algorithmic bytes per launch = N x (K x 81 + 224)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 65536


def avg(path, counter, kernel="env_rollout"):
    """Mean counter value over the matching dispatches of the largest grid
    (bench.py's host-floor probe launches the same kernel on 64 envs)."""
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    big = max((g for g, _ in rows), default=0)
    vals = [v for g, v in rows if g == big]
    if not vals:
        raise SystemExit(f"no {counter} rows under {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    out = sys.argv[1]
    tj_path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(tj_path))
    for k in (32, 20):
        f, nf = avg(os.path.join(out, f"k{k}_FETCH_SIZE"), "FETCH_SIZE")
        w, nw = avg(os.path.join(out, f"k{k}_WRITE_SIZE"), "WRITE_SIZE")
        rd, wr = f * 2048, w * 1024
        tj[f"rollout_f64_{N}_k{k}"] = {
            "algorithmic_bytes_per_launch": N * (k * 81 + 224),
            "hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd),
            "write_bytes": round(wr), "dispatches": [nf, nw],
            "source": "scripts/rollout_traffic.sh (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE "
                      "passes; FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, KiB -> B)"}
        print(k, json.dumps(tj[f"rollout_f64_{N}_k{k}"]))
    # the companion: 4,194,304 envs, K = 32, the one-role kernel (the headline
    # at 65,536 envs runs the warp-specialised forms, other kernel names)
    n4, k = 1 << 22, 32
    if os.path.isdir(os.path.join(out, "c4m_FETCH_SIZE")):
        f, nf = avg(os.path.join(out, "c4m_FETCH_SIZE"), "FETCH_SIZE", "env_rollout_kernel")
        w, nw = avg(os.path.join(out, "c4m_WRITE_SIZE"), "WRITE_SIZE", "env_rollout_kernel")
        rd, wr = f * 2048, w * 1024
        tj[f"rollout_f64_{n4}_k{k}"] = {
            "algorithmic_bytes_per_launch": n4 * (k * 81 + 224),
            "hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd),
            "write_bytes": round(wr), "dispatches": [nf, nw],
            "source": "scripts/rollout_traffic.sh companion passes (bench.py's "
                      "companion_rollout; rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE; FETCH_SIZE "
                      "x2 gfx950 correction + WRITE_SIZE, KiB -> B)"}
        print("companion", json.dumps(tj[f"rollout_f64_{n4}_k{k}"]))
    json.dump(tj, open(tj_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
