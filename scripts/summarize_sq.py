"""SQ counters of the fused kernel (scripts/gpu_pmc_sq.sh output, gpurun_out/sq/p*) -> one JSON:
per-launch averages, per wave per step instruction counts and the share of wave time spent
waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES; both in quad-cycles, MI355X_MICROARCH.md).

usage: python scripts/summarize_sq.py <out.json> [--epw 16] [--envs 4096] [--steps 200]
"""
import argparse
import collections
import csv
import glob
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out", "sq"))
ap.add_argument("--epw", type=int, default=16)
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
grid = (a.envs + a.epw - 1) // a.epw * 512
vals = collections.defaultdict(dict)          # (pass, dispatch) -> counter -> value
for path in glob.glob(os.path.join(a.src, "p*", "*counter_collection.csv")):
    tag = os.path.basename(os.path.dirname(path))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if not (name == "k_step_ag" or name.startswith("k_step_ag<")) or int(row["Grid_Size"]) != grid:
                continue
            d = vals[(tag, row["Dispatch_Id"])]
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
per = collections.defaultdict(list)
for d in vals.values():
    for k, v in d.items():
        per[k].append(v)
avg = {k: sum(v) / len(v) for k, v in per.items()}
waves = avg.get("SQ_WAVES", grid / 64)
ws = waves * a.steps
out = {"kernel": "k_step_ag<lds,predraw>", "envs_per_workgroup": a.epw,
       "launch": f"{a.envs} envs x {a.steps} steps", "launches_per_counter": {k: len(v) for k, v in per.items()},
       "per_launch_avg": avg,
       "per_wave_per_step": {"VALU": avg.get("SQ_INSTS_VALU", 0) / ws, "SALU": avg.get("SQ_INSTS_SALU", 0) / ws,
                             "LDS": avg.get("SQ_INSTS_LDS", 0) / ws,
                             "wave_cycles": 4 * avg.get("SQ_WAVE_CYCLES", 0) / ws},
       "wait_share": avg.get("SQ_WAIT_ANY", 0) / max(1.0, avg.get("SQ_WAVE_CYCLES", 1)),
       "issue_stall_share": avg.get("SQ_WAIT_INST_ANY", 0) / max(1.0, avg.get("SQ_WAVE_CYCLES", 1)),
       "active_share": avg.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, avg.get("SQ_WAVE_CYCLES", 1)),
       "note": "rocprofv3 --pmc, one pass per group (scripts/gpu_pmc_sq.sh); SQ_WAVE_CYCLES / SQ_WAIT_* / "
               "SQ_ACTIVE_* in quad-cycles; wait = s_waitcnt / barrier / s_sleep parked"}
with open(a.out, "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
