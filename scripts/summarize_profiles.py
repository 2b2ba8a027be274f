"""Turn the rocprofv3 output of scripts/gpu_profile.sh (gpurun_out/prof) into the committed
evidence under profiles/: copies of the stats / trace / counter CSVs for round ROUND, the
per-launch HBM traffic JSON bench.py reads (profiles/pmc_<workload>.json) and a short summary.

usage: python scripts/summarize_profiles.py r01 [--envs 4096] [--steps-per-launch 1000]

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE
and WRITE_SIZE are kB; FETCH_SIZE counts half of a wide streaming read on gfx950, so reads are
doubled (an upper bound for this kernel's narrow gathers); each counter has its own pass.
"""
import argparse
import csv
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, kernel, grid):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Kernel_Name"].startswith(kernel) and int(row["Grid_Size"]) % grid == 0 and int(row["Grid_Size"]) <= 16 * grid:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out", "prof"))
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps-per-launch", type=int, default=1000)
    ap.add_argument("--kernel", default="k_step_ag")
    ap.add_argument("--variant", default="k_step_ag<lds,predraw>", help="fjsp_last_kernel name of the profiled launch")
    ap.add_argument("--algo-bytes-per-env-step", type=int, default=211)
    a = ap.parse_args()
    dst = os.path.join(REPO, "profiles", a.round)
    os.makedirs(dst, exist_ok=True)
    tag = f"bench{a.envs}"
    copies = {
        "kt/kt_kernel_stats.csv": f"kernel_stats_{tag}.csv",
        "kt/kt_kernel_trace.csv": f"kernel_trace_{tag}.csv",
        "fetch/fetch_counter_collection.csv": "pmc_fetch_size.csv",
        "write/write_counter_collection.csv": "pmc_write_size.csv",
    }
    for s, d in copies.items():
        shutil.copyfile(os.path.join(a.src, s), os.path.join(dst, d))
    grid = a.envs if a.envs % 64 == 0 else (a.envs + 63) // 64 * 64
    fetch = per_kernel(os.path.join(a.src, copies_src("fetch")), a.kernel, grid)
    write = per_kernel(os.path.join(a.src, copies_src("write")), a.kernel, grid)
    if not fetch or not write:
        raise SystemExit(f"no {a.kernel} launches with grid {grid} in the counter CSVs")
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    hbm = (2.0 * fk + wk) * 1024.0
    algo = a.algo_bytes_per_env_step * a.envs * a.steps_per_launch
    stats = {}
    with open(os.path.join(a.src, "kt/kt_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = row
    k = stats.get(a.kernel, {})
    rel = os.path.relpath(dst, REPO)
    pmc = {
        "workload": f"fjsp_step_{a.envs}envs",
        "envs": a.envs,
        "steps_per_launch": a.steps_per_launch,
        "kernel": a.kernel,
        "kernel_variant": a.variant,
        "launches": len(fetch),
        "FETCH_SIZE_kB_per_launch": fk,
        "WRITE_SIZE_kB_per_launch": wk,
        "hbm_bytes_per_launch": hbm,
        "algo_bytes_per_launch": algo,
        "hbm_over_algo": hbm / algo,
        "rocprof_avg_launch_ns": float(k["AverageNs"]) if k else None,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                  "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md (FETCH_SIZE "
                  "reads 1/2 of a wide streaming read on gfx950; doubling is an upper bound for "
                  "this kernel's narrow gathers)",
        "source": f"{rel}/pmc_fetch_size.csv, {rel}/pmc_write_size.csv, {rel}/kernel_stats_{tag}.csv",
    }
    with open(os.path.join(REPO, "profiles", f"pmc_fjsp_step_{a.envs}envs.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    print(json.dumps(pmc, indent=1))


def copies_src(which):
    return f"{which}/{which}_counter_collection.csv"


if __name__ == "__main__":
    main()
