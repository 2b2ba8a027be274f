"""Turn the rocprofv3 output of scripts/gpu_profile.sh (gpurun_out/prof) into the committed
evidence under profiles/: copies of the stats / trace / counter CSVs for round ROUND, and one
HBM-traffic JSON per profiled step kernel that bench.py reads
(profiles/pmc_<workload>.json, keyed per env-step so it applies to any launch length):

  * fjsp_step_<envs>envs  - the fused kernel of the headline (k_step_ag), full-length launches
  * k_step_<envs>envs     - the one-launch-per-step kernel (reference-API / A2C collect path)

usage: python scripts/summarize_profiles.py r02 [--envs 4096] [--steps-per-launch 1024]

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE
and WRITE_SIZE are kB, each counter has its own pass; FETCH_SIZE counts half of a wide streaming
read on gfx950, so reads are doubled (an upper bound for these kernels' narrow gathers).
"""
import argparse
import csv
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def launches(path, kernel, grid):
    """[(counter kB, duration ns)] of the launches of `kernel` (exact name) with this grid."""
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if (name == kernel or name.startswith(kernel + "<")) and int(row["Grid_Size"]) == grid:
                out.append((float(row["Counter_Value"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    return out


def full(ls, steps_per_launch):
    """Multi-step launches: the full-length ones (a trailing shorter chunk is dropped).
    One-step launches: every launch after the first 20 (cold caches / first-touch)."""
    if steps_per_launch == 1:
        return [v for v, _ in ls[20:]] or [v for v, _ in ls]
    m = max(d for _, d in ls)
    return [v for v, d in ls if d >= 0.8 * m]


def summarize(a, dst, kernel, variant, grid, workload, steps_per_launch, algo_per_env_step, stats, rel):
    fetch = full(launches(os.path.join(a.src, "fetch/fetch_counter_collection.csv"), kernel, grid), steps_per_launch)
    write = full(launches(os.path.join(a.src, "write/write_counter_collection.csv"), kernel, grid), steps_per_launch)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} launches with grid {grid} in the counter CSVs")
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    hbm = (2.0 * fk + wk) * 1024.0
    env_steps = a.envs * steps_per_launch
    algo = algo_per_env_step * env_steps
    k = next((v for n, v in stats.items() if n == kernel or n.startswith(kernel + "<")), {})
    # kernel-trace durations of the same launches (the stats' average mixes in shorter launches)
    tr = []
    with open(os.path.join(a.src, "kt/kt_kernel_trace.csv")) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if (name == kernel or name.startswith(kernel + "<")) and int(row["Grid_Size_X"]) == grid:
                tr.append((0.0, int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    durs = [d for _, d in tr]
    if steps_per_launch == 1:
        durs = durs[20:] or durs
    else:
        durs = [d for d in durs if d >= 0.8 * max(durs)] if durs else []
    avg_full = sum(durs) / len(durs) if durs else None
    pmc = {
        "workload": workload,
        "envs": a.envs,
        "steps_per_launch": steps_per_launch,
        "kernel": kernel,
        "kernel_variant": variant,
        "launches": [len(fetch), len(write)],
        "FETCH_SIZE_kB_per_launch": fk,
        "WRITE_SIZE_kB_per_launch": wk,
        "hbm_bytes_per_launch": hbm,
        "hbm_bytes_per_env_step": hbm / env_steps,
        "algo_bytes_per_env_step": algo_per_env_step,
        "algo_bytes_per_launch": algo,
        "hbm_over_algo": hbm / algo,
        "rocprof_avg_launch_ns_all": float(k["AverageNs"]) if k else None,
        "rocprof_avg_launch_ns_full": avg_full,
        "rocprof_full_launches": len(durs),
        "achieved_GBs_full": algo / avg_full if avg_full else None,
        "frac_of_8TBs_full": algo / avg_full / 8000.0 if avg_full else None,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                  "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md (FETCH_SIZE "
                  "reads 1/2 of a wide streaming read on gfx950; doubling is an upper bound for "
                  "these kernels' narrow gathers); full-length launches only",
        "source": f"{rel}/pmc_fetch_size.csv, {rel}/pmc_write_size.csv, {rel}/kernel_stats_bench{a.envs}.csv",
    }
    with open(os.path.join(REPO, "profiles", f"pmc_{workload}.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    return pmc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out", "prof"))
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps-per-launch", type=int, default=1024)
    ap.add_argument("--variant", default="k_step_ag<lds,predraw>", help="fjsp_last_kernel name of the fused launch")
    ap.add_argument("--epw", type=int, default=16, help="k_step_ag envs per workgroup (option ag_envs; auto at 4096 envs: 16)")
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
    stats = {}
    with open(os.path.join(a.src, "kt/kt_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = row
    rel = os.path.relpath(dst, REPO)
    grid_ag = (a.envs + a.epw - 1) // a.epw * 64 * 8   # k_step_ag: 8 waves per workgroup of epw envs
    grid_1 = (a.envs + 63) // 64 * 64
    out = {
        "fused": summarize(a, dst, "k_step_ag", a.variant, grid_ag, f"fjsp_step_{a.envs}envs", a.steps_per_launch,
                           211, stats, rel),
        "per_step": summarize(a, dst, "k_step", "k_step<canon>", grid_1, f"k_step_{a.envs}envs", 1, 219, stats, rel),
    }
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
