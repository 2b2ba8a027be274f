#!/usr/bin/env python3
"""Summarise the A2C bench's rocprofv3 passes (scripts/gpu.sh <out> prof_a2c: gpurun_out/<out>/a2c_{kt,
fetch_size,write_size,tcc_hit_sum}) into profiles/<round>/a2c/: the kernel stats CSV and pmc_collect_summary.json,
per kernel: launches, average duration, HBM bytes per launch ((2 x FETCH_SIZE + WRITE_SIZE) kB,
MI355X_MICROARCH.md's gfx950 correction), per env, against the algorithmic bytes, and the L2 hit
rate (TCC_HIT / (TCC_HIT + TCC_MISS)).

usage: python scripts/summarize_a2c.py r04 [--envs 4096]"""
import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# split-bf16 packed weights read once per launch (include/fjsp.h FJSP_POLICY_*_FLOATS)
ACTOR_FLOATS = 3 * 256 * 16 // 2 + 256 + 3 * 256 * 256 // 2 + 256 + 8 * 256 + 16
CRITIC_FLOATS = 3 * 256 * 48 // 2 + 256 + 3 * 256 * 256 // 2 + 256 + 3 * 128 * 256 // 2 + 128 + 128 + 16
WEIGHT_BYTES = 4 * (8 * ACTOR_FLOATS + CRITIC_FLOATS)
# per env of one launch: in = features 152 B + masks 29 B; policy out = actions 8 + value 4; step out =
# next features 152 + next masks 29 + rewards 64 + term/trunc 2 + status 4 (the 8 action bytes of the
# tile hand-off are written and read once more)
ALGO = {"k_policy_step": 152 + 29 + 8 + 4 + 152 + 29 + 64 + 2 + 4,
        "k_policy": 152 + 29 + 8 + 4,
        "k_step": 8 + 152 + 29 + 64 + 2 + 4}
WEIGHTS = {"k_policy_step": WEIGHT_BYTES, "k_policy": WEIGHT_BYTES}


def short(name):
    return name.split("(")[0].split("<")[0].replace("(anonymous namespace)::", "").strip()


def counters(path):
    """kernel -> [(value, grid)] from a rocprofv3 counter-collection CSV (one counter per pass)."""
    out = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            out[(short(row["Kernel_Name"]), row["Counter_Name"])].append(float(row["Counter_Value"]))
    return out


def find(base, suffix):
    for root, _, files in os.walk(base):
        for fn in files:
            if fn.endswith(suffix):
                return os.path.join(root, fn)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--src", required=True, help="gpurun_out/<out> of a `scripts/gpu.sh <out> prof_a2c` run")
    a = ap.parse_args()
    dst = os.path.join(REPO, "profiles", a.round, "a2c")
    os.makedirs(dst, exist_ok=True)
    stats = {}
    sp = find(os.path.join(a.src, "a2c_kt"), "kernel_stats.csv")
    with open(sp) as f:
        for row in csv.DictReader(f):
            stats[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                         "total_ns": float(row["TotalDurationNs"]),
                                         "pct": float(row["Percentage"])}
    shutil.copy(sp, os.path.join(dst, f"kernel_stats_a2c{a.envs}.csv"))
    c = {}
    for p in ("fetch_size", "write_size", "tcc_hit_sum"):
        f = find(os.path.join(a.src, "a2c_" + p), "counter_collection.csv")
        if f:
            c.update(counters(f))
    res = {"workload": f"bench.py --workload a2c ({a.envs} envs, batch 256), kernel trace + separate PMC passes",
           "method": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (MI355X_MICROARCH.md); "
                     "L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS); averages over every launch of the kernel",
           "kernels": {}}
    for k in ("k_policy_step", "k_policy", "k_step", "k_gae", "k_critic_fwd", "k_critic_bwd", "k_group_keys",
              "k_group_verify", "k_actor_head", "k_value_head_grad"):
        if k not in stats:
            continue
        e = {"calls": stats[k]["calls"], "avg_us": stats[k]["avg_ns"] / 1e3, "pct_of_kernel_time": stats[k]["pct"]}
        fe, wr = c.get((k, "FETCH_SIZE")), c.get((k, "WRITE_SIZE"))
        if fe and wr:
            fk, wk = sum(fe) / len(fe), sum(wr) / len(wr)
            e["FETCH_SIZE_kB_per_launch"], e["WRITE_SIZE_kB_per_launch"] = fk, wk
            e["hbm_bytes_per_launch"] = (2 * fk + wk) * 1024
            if k in ALGO:
                algo = ALGO[k] * a.envs + WEIGHTS.get(k, 0)
                e["algo_bytes_per_launch"] = algo
                e["hbm_bytes_per_env"] = e["hbm_bytes_per_launch"] / a.envs
                e["hbm_over_algo"] = e["hbm_bytes_per_launch"] / algo
        hi, mi = c.get((k, "TCC_HIT_sum")), c.get((k, "TCC_MISS_sum"))
        if hi and mi:
            e["l2_hit_rate"] = sum(hi) / max(1.0, sum(hi) + sum(mi))
        res["kernels"][k] = e
    res["weights_bytes_split_bf16"] = WEIGHT_BYTES
    with open(os.path.join(dst, "pmc_collect_summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
