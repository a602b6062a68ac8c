"""Copy this round's rocprofv3 counter passes from gpurun_out/<tag>/ into
profiles/ and record, in profiles/<tag>_pmc_manifest.json, the libmpcr.so
source hash of the build they were taken from (manipulator_mujoco_amd.build
.source_hash) -- bench.py attaches committed counters only to a run of that
same build.  The hash is the one the session itself recorded
(gpurun_out/<tag>/source_hash.txt, tools/gpu_session_r05.sh); the script
refuses to commit when the checkout no longer hashes to it (an
edit between the session and this script would attach the counters to a
build they were not taken from).

    python tools/commit_profiles.py r05
"""
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from manipulator_mujoco_amd import build  # noqa: E402

# session pass directory -> committed name (bench.py: <tag>_pmc_<kind><suffix>.csv)
PASSES = {"pmc1": "pmc_rollout_fetch", "pmc2": "pmc_rollout_write", "pmc3": "pmc_sq",
          "pmc_c2_FETCH_SIZE": "pmc_rollout_fetch_c2", "pmc_c2_WRITE_SIZE": "pmc_rollout_write_c2",
          "pmc_c2_sq": "pmc_sq_c2", "pmc_c4_FETCH_SIZE": "pmc_rollout_fetch_c4",
          "pmc_c4_WRITE_SIZE": "pmc_rollout_write_c4", "pmc_c4": "pmc_sq_c4"}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
    src = os.path.join(ROOT, "gpurun_out", tag)
    man_path = os.path.join(ROOT, "profiles", f"{tag}_pmc_manifest.json")
    man = json.load(open(man_path)) if os.path.exists(man_path) else {}
    h = build.source_hash()
    hf = os.path.join(src, "source_hash.txt")
    if not os.path.exists(hf):
        sys.exit(f"{hf} missing: the session did not record the build it ran")
    ran = open(hf).read().strip()
    if ran != h:
        sys.exit(f"the session ran build {ran}, the checkout is {h}: not committing its counters")
    merged = {}
    for d, name in PASSES.items():
        f = os.path.join(src, d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        kind = name.replace("_fetch", "").replace("_write", "")
        merged.setdefault(kind, []).append(f)
    for kind, files in merged.items():
        out = os.path.join(ROOT, "profiles", f"{tag}_{kind}.csv")
        with open(out, "w") as fo:
            for i, f in enumerate(files):  # FETCH and WRITE passes into one CSV (one header)
                lines = open(f).read().splitlines(True)
                fo.writelines(lines if i == 0 else lines[1:])
        man[os.path.basename(out)] = {"source_hash": h, "passes": [os.path.relpath(f, ROOT) for f in files],
                                      "recorded": time.strftime("%Y-%m-%d %H:%M:%S")}
        print(out)
    json.dump(man, open(man_path, "w"), indent=1)
    print(man_path, h)


if __name__ == "__main__":
    main()
