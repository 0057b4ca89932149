"""Record which kernel sources a committed profile was measured on.

    python scripts/provenance.py record profiles/r05_kernel_stats.csv ...
        stamp the named profiles with this tree's kernel_source_hash (run
        right after copying a GPU session's results into profiles/, before
        any kernel source changes)
    python scripts/provenance.py backfill profiles/r04_kernel_stats.csv ...
        stamp each named profile with the hash of the kernel sources at the
        commit that last changed that profile (git show, no checkout)
    python scripts/provenance.py check
        list every entry and whether it matches the current tree

bench.py reads profiles/provenance.json (committed_profile) and reports a
committed number inside a live block only when its hash equals the current
tree's; otherwise it goes to the line's committed_artefacts block, stale.
Runs here (CPU), never on the GPU box.
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

PROV = bench.PROVENANCE_JSON


def _load():
    try:
        return json.load(open(PROV))
    except (OSError, ValueError):
        return {}


def _save(d):
    with open(PROV, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
        f.write("\n")


def _git(*a):
    return subprocess.run(["git", "-C", ROOT] + list(a), check=True, capture_output=True,
                          text=True).stdout


def hash_at(commit):
    """kernel_source_hash() of the tree at `commit` (same file set and order)."""
    names = sorted(os.path.basename(p) for p in
                   _git("ls-tree", "--name-only", commit, "drone_rl_amd/csrc/").split())
    files = [f for f in names if f.endswith((".hip", ".h")) or f == "Makefile"]
    h = hashlib.sha256()
    for rel in [f"drone_rl_amd/csrc/{f}" for f in files] + ["include/dronerl.h"]:
        data = subprocess.run(["git", "-C", ROOT, "show", f"{commit}:{rel}"], check=True,
                              capture_output=True).stdout
        h.update(rel.encode() + b"\0")
        h.update(data)
        h.update(b"\0")
    return h.hexdigest()


def main():
    cmd, paths = sys.argv[1], sys.argv[2:]
    d = _load()
    if cmd == "record":
        cur = bench.kernel_source_hash()
        head = _git("rev-parse", "--short", "HEAD").strip()
        for p in paths:
            d[os.path.basename(p)] = {"source_hash": cur, "recorded_at_head": head}
        _save(d)
    elif cmd == "backfill":
        for p in paths:
            c = _git("log", "-1", "--format=%h", "--", os.path.relpath(p, ROOT)).strip()
            d[os.path.basename(p)] = {"source_hash": hash_at(c), "recorded_at_head": c}
        _save(d)
    elif cmd == "check":
        cur = bench.kernel_source_hash()
        for k, v in sorted(d.items()):
            print(f"{k:40s} {v['source_hash'][:12]} {'MATCH' if v['source_hash'] == cur else 'stale'}")
    else:
        sys.exit(f"unknown command {cmd}")


if __name__ == "__main__":
    main()
