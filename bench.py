#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the vectorised FJSP step on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the metric's "4096 parallel envs on 1 MI355X"): 4096
reference environments per GPU (num_orders=30, default CONFIG), synthetic uniformly random
actions (action_space.sample() semantics) from the on-device counter RNG, auto-reset on
truncation/termination (MT19937 stream continued like reset(seed=None)).  One bench "step" =
one rollout batch: --batch-steps (default 256, the reference's A2C batch / rollout horizon,
train.py:59 --batch_size 256) consecutive FJSPSimulation.step() calls of every env on this GPU,
i.e. 256 x 4096 env-steps; obs (reference dtypes), fp64 rewards, term and trunc of every
env-step are written to an HBM trajectory slab.  The env-steps of the timed region are
executed by the fused step kernel in launches of --chunk env-steps; the variant launched is
reported in config.kernel.  value = env-steps per second (BASELINE.json's metric).

Multi-GPU (torchrun): one process per GPU, envs sharded by global id (rank * envs + e) with
no data-path collective ("scaling": "weak"); the only collectives are the barrier and the
max-over-ranks of the elapsed time.

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import importlib
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ALGO_BYTES_FUSED = 145 + 64 + 2          # obs (reference dtypes) + f64 rewards[8] + term + trunc
ALGO_BYTES_STEP = 8 + ALGO_BYTES_FUSED   # + u8 actions[8] read from HBM
HBM_PEAK_GBS = 8000.0                     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Under torch.distributed.run it must equal WORLD_SIZE; "
                         "without it, N > 1 starts N rank processes itself (launch_ranks)")
    ap.add_argument("--steps", type=int, default=None, help="bench steps: default 20 rollout batches (step) / 4 A2C batches (a2c)")
    ap.add_argument("--warmup", type=int, default=None, help="default 5 rollout batches (step) / 3 A2C batches (a2c)")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--batch-steps", type=int, default=256,
                    help="env-steps of every env per bench step (one rollout batch, train.py:59)")
    ap.add_argument("--chunk", type=int, default=1024,
                    help="env steps per fused launch (also timed at 200 per launch: chunk_200 in the JSON)")
    ap.add_argument("--no-chunk-compare", action="store_true", help="skip the 200-step-launch comparison")
    ap.add_argument("--num-orders", type=int, default=30)
    ap.add_argument("--masked", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="wall budget of each CPU baseline leg (single thread, all cores)")
    ap.add_argument("--no-step-mode", action="store_true", help="skip the one-launch-per-step measurement")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the host-driven legs: the reference-API (FJSPParallelEnv.step, one env) latency and "
                         "the host-action vector step (launch path and step server)")
    ap.add_argument("--workload", choices=["step", "a2c"], default="step",
                    help="step: env-step throughput (the headline metric); a2c: the batched A2C "
                         "training loop (BASELINE configs 4/5; one bench step = one A2C batch)")
    ap.add_argument("--batch-size", type=int, default=256, help="A2C batch (vector steps per update)")
    ap.add_argument("--no-a2c", action="store_true", help="skip the A2C training-loop leg of the step workload")
    ap.add_argument("--no-scale", action="store_true", help="skip the 16x-envs leg of the step workload")
    ap.add_argument("--no-dedup", action="store_true",
                    help="A2C update over every sample (no grouping of repeated inputs)")
    ap.add_argument("--exchange", choices=["allreduce", "gather", "shard"], default="shard",
                    help="a2c workload with several ranks: the once-per-batch exchange (shard = the experience "
                         "routed to the rank that learns from it: combined records in one all_to_all, actor a on "
                         "rank a, critic states by key, shard_learner.py; gather = the transition slabs into "
                         "rank 0, the serial learner of a2c.py:324-336; allreduce = one flat gradient all_reduce)")
    ap.add_argument("--init", choices=["random", "trained"], default="random",
                    help="a2c workload: random-init networks or the reference's trained checkpoint")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = 20 if a.workload == "step" else 4
    if a.warmup is None:
        a.warmup = 5 if a.workload == "step" else 3
    return a


def host_cores():
    """(threads to use, description): the CPUs this process may run on, capped by the cgroup
    CPU quota when one is set (a GPU box shows the whole machine's CPUs in nproc / affinity but
    grants one GPU's share)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except Exception:
        pass
    use = min(aff, quota) if quota else aff
    return use, {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota}


def cpu_baseline(args):
    """The oracle (C restatement of the reference step with a SimPy event heap, kind='port') on
    the host: one thread, then one thread per available core (env shards), bounded samples of
    the same workload (random-action rollouts, auto-reset)."""
    from oracle import oracle as O
    O.lib()
    steps = 200
    t0 = time.perf_counter()
    O.rollout(16, steps, num_orders=args.num_orders, record=False)
    per_env_step = (time.perf_counter() - t0) / (16 * steps)
    envs_per_thread = max(1, int(args.cpu_seconds / (per_env_step * steps)))

    def leg(workers):
        def work(i):
            O.rollout(envs_per_thread, steps, seeds=np.arange(i * envs_per_thread, (i + 1) * envs_per_thread),
                      gid0=i * envs_per_thread, num_orders=args.num_orders, record=False,
                      policy=1 if args.masked else 0)

        th = [threading.Thread(target=work, args=(i,)) for i in range(workers)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        return workers * envs_per_thread * steps / wall, wall

    v1, w1 = leg(1)
    cores, info = host_cores()
    vn, wn = leg(cores)
    return {"value": vn, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "value_1thread": v1,
            "sample": f"{envs_per_thread} envs x {steps} steps per thread of the same workload (oracle/fjsp_oracle.c, "
                      f"C restatement of FJSPSimulation.step with a SimPy event heap): 1 thread {w1:.1f}s wall, "
                      f"{cores} threads (one per available core) {wn:.1f}s wall",
            "host": info,
            "reference_python_1core": "8.0-9.0k env-steps/s (measured in the build container, BASELINE.md)"}


REF_PY_STEP_US = 115.0   # the reference FJSPSimulation.step, 1 core (112.9-115.6 us)


def dropin_latency(dev, steps=2000, warm=200):
    """The reference-API path a2c.py drives (a2c.py:294-305): one FJSPParallelEnv.step(dict) per
    Python iteration on ONE env, then the visualiser's reads of simulation.agv.position and
    agv.carrying_tray, the episode restarted with reset() when env.agents empties (the loop's
    `while self.env.agents`).  Wall time per call on this host, beside the reference's ~115 us.
    Also: the same without the agv reads, the same through one launch + one synchronisation per
    step instead of the step server, and one server request alone."""
    W = importlib.import_module("multi-agent-rl-for-fjsp_amd.FJSPParallelEnvWrapper")
    env = W.FJSPParallelEnv()
    env.reset(seed=0, options={"num_orders": 30})
    rng = np.random.default_rng(0)
    n_act = [env.action_space(a).n for a in env.possible_agents]
    acts = [{a: int(rng.integers(0, n_act[i])) for i, a in enumerate(env.possible_agents)} for _ in range(steps)]
    sim = env.unwrapped.simulation

    def loop(agv_reads, n):
        resets = 0
        t0 = time.perf_counter()
        for t in range(n):
            env.step(acts[t])
            if agv_reads:
                _ = sim.agv.position
                _ = sim.agv.carrying_tray is not None
            if not env.agents:
                env.reset(options={"num_orders": 30})
                resets += 1
        return (time.perf_counter() - t0) / n * 1e6, resets

    loop(True, warm)
    with_agv, resets = loop(True, steps)
    no_agv, _ = loop(False, steps)
    # the same loop through one launch + one synchronisation per step (the step server off)
    sim.use_server = False
    loop(True, warm)
    launch_path, _ = loop(True, steps)
    sim.use_server = True
    # the device part alone: one server request (doorbell + wait) on the facade's record, in the
    # facade's inline mode (the action bytes in the doorbell's line) and with an actions buffer
    L, h = sim._L, sim._h
    nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
    env.reset(seed=1, options={"num_orders": 30})

    def requests(inline):
        nat.check(L.fjsp_server_start(h, None if inline else sim._act_ptr, 0, sim._packed.ref_full))
        req = (lambda: L.fjsp_server_step_actions(h, sim._act_ptr)) if inline else (lambda: L.fjsp_server_step(h))
        for _ in range(100):
            nat.check(req())
        t0 = time.perf_counter()
        for _ in range(steps):
            nat.check(req())
        us = (time.perf_counter() - t0) / steps * 1e6
        nat.check(L.fjsp_server_stop(h))
        return us
    server_buf_us = requests(False)
    server_us = requests(True)   # leaves the facade's own configuration behind
    return {"dropin_n1_us_per_step": with_agv, "dropin_n1_no_agv_reads_us_per_step": no_agv,
            "dropin_n1_launch_path_us_per_step": launch_path, "server_request_us": server_us,
            "server_request_actions_buffer_us": server_buf_us,
            "resets": resets, "steps": steps,
            "reference_us_per_step": REF_PY_STEP_US,
            "speedup_vs_reference": REF_PY_STEP_US / with_agv,
            "note": "FJSPParallelEnv.step(dict) + a2c.py:298-305's agv.position / carrying_tray reads, one env, "
                    "random actions, reset when env.agents empties; the step server carries the canonical-order "
                    "steps (launch_path: one fjsp_step launch + one synchronisation per step instead); "
                    "server_request_us: one fjsp_server_step_actions alone (inline mode, the facade's), "
                    "server_request_actions_buffer_us: one fjsp_server_step reading an actions buffer; reference: SURVEY.md App. E (1 core, same "
                    "container class), not re-timed on this box (the reference never travels)"}


def host_action_step(env, dev, N, K=200):
    """FJSPVecEnv.step with actions handed over from HOST memory each step (a CPU-side policy):
    pinned u8[8][N] -> H2D -> k_step -> outputs in HBM, one synchronisation per step; and the
    same with the step's lean outputs (obs, masks, rewards, term, trunc) copied back to host."""
    vec_env = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
    nact = np.array([3, 8, 3, 3, 3, 3, 3, 3], np.int64).reshape(8, 1)
    rng = np.random.default_rng(1)
    host = [torch.from_numpy(((rng.integers(0, 256, (8, N)) * nact) >> 8).astype(np.uint8)).pin_memory()
            for _ in range(K)]
    sbuf = vec_env.Buffers(1, N, dev, infos=False)
    back = {k: torch.empty(getattr(sbuf, k).shape, dtype=getattr(sbuf, k).dtype).pin_memory()
            for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc")}

    def run(copy_back):
        t0 = time.perf_counter()
        for t in range(K):
            env.step(host[t], buffers=sbuf)
            if copy_back:
                for k, h in back.items():
                    h.copy_(getattr(sbuf, k), non_blocking=True)
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e6

    run(False)
    a = run(False)
    b = run(True)
    # the same through the step server: the actions rewritten in one pinned buffer before every
    # step, one doorbell per step, no launch and no stream synchronisation
    srv = torch.zeros(8, N, dtype=torch.uint8).pin_memory()
    env.server_start(srv, autoreset=True, buffers=sbuf)
    for t in range(20):
        srv.copy_(host[t])
        env.server_step()
    t0 = time.perf_counter()
    for t in range(K):
        srv.copy_(host[t])
        env.server_step()
    c = (time.perf_counter() - t0) / K * 1e6
    env.server_stop()
    # and with the step's outputs written by the server straight into pinned host memory (what a
    # CPU-side policy reads next), no copy call
    hbuf = vec_env.Buffers(1, N, "cpu", infos=False)
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status"):
        setattr(hbuf, k, getattr(hbuf, k).pin_memory())
    env.server_start(srv, autoreset=True, buffers=hbuf)
    for t in range(20):
        srv.copy_(host[t])
        env.server_step()
    t0 = time.perf_counter()
    for t in range(K):
        srv.copy_(host[t])
        env.server_step()
    d = (time.perf_counter() - t0) / K * 1e6
    env.server_stop()
    return {"envs": N, "us_per_step": a, "value": N / (a * 1e-6), "unit": "env-steps/s",
            "us_per_step_with_outputs_to_host": b, "value_with_outputs_to_host": N / (b * 1e-6),
            "server_us_per_step": c, "server_value": N / (c * 1e-6),
            "server_us_per_step_outputs_to_host": d, "server_value_outputs_to_host": N / (d * 1e-6),
            "note": "actions from pinned host memory every step (H2D + k_step + sync); the second figure also "
                    "copies obs/masks/rewards/term/trunc back to pinned host memory; server_*: the same steps "
                    "through the step server (fjsp_server_step: resident kernel, host doorbell), outputs in HBM "
                    "or (outputs_to_host) written by the kernel into pinned host memory"}


def load_pmc(workload):
    p = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f)
    except Exception:
        return None


TRAINED_NPZ = os.path.join(REPO, "tests", "golden", "trained_policy.npz")


def a2c_throughput(env, N, world, batches, warmup, batch_size, num_orders, dist=None, group=None, dedup=True,
                   exchange="allreduce", init="random", stats=True):
    """Batched A2C training loop (a2c_vec.VecMultiAgentA2C): env-steps/s over whole batches
    (collect batch_size vector steps with the policy + GAE + one update).  dedup: the update
    runs each network once per distinct input (A2CLosses; the same gradient).  exchange: the
    multi-rank exchange ("shard": combined records to the rank owning each network, one
    all_to_all + one gradient all_reduce; "allreduce" of gradients; "gather" of the transition
    slabs into rank 0, a2c.py:324-336).  init "trained": start from the reference's trained checkpoint
    (checkpoints/model.pt, carried as tests/golden/trained_policy.npz)."""
    A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    learner = A.VecMultiAgentA2C(env, batch_size=batch_size, seed=0, group=group, dedup=dedup, exchange=exchange)
    if init == "trained":
        learner.load_state_dicts(A.load_npz_weights(TRAINED_NPZ))
    base = env.env_id_base
    learner.reset(seeds=torch.arange(base, base + N), num_orders=num_orders)

    def batch():
        learner.collect()
        learner.update()
        learner.roll_over()
    for _ in range(warmup):
        batch()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    tc = 0.0
    for _ in range(batches):
        c0 = time.perf_counter()
        learner.collect()
        torch.cuda.synchronize()
        tc += time.perf_counter() - c0
        learner.update()
        learner.roll_over()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    check_faults(env)
    if dist:
        t = torch.tensor([elapsed, tc], device=env.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, tc = float(t[0]), float(t[1])
    steps = batches * batch_size * N * world
    out = {"value": steps / elapsed, "unit": "env-steps/s", "n_gpus": world, "batches": batches,
           "batch_size": batch_size, "envs_per_gpu": N, "ms_per_batch": elapsed * 1e3 / batches,
           "collect_ms_per_batch": tc * 1e3 / batches,
           "update_ms_per_batch": (elapsed - tc) * 1e3 / batches,
           "critic_loss_last": learner.critic_loss_history[-1], "update_dedup": bool(dedup),
           "exchange": exchange if world > 1 else None, "init": init,
           "note": "collect = one k_policy_step launch per vector step and env group (fused MFMA predict + "
                   "the env step of each 64-env tile, features and masks written in HBM; two env-group streams) -> "
                   "fp64 GAE kernel -> grouped full-batch update (8 actors + critic, Adam); reference a2c.py "
                   "loop: ~130 env-steps/s on one CPU core (SURVEY.md)"}
    if world > 1:
        grad_bytes = 4 * sum(p.numel() for p in list(learner.actors.parameters()) + list(learner.critic.parameters()))
        if exchange == "gather":
            out["exchange_bytes_per_rank_per_batch"] = learner.exchange_bytes_per_batch()
        elif exchange == "shard":
            # the last batch's records sent to the other ranks (measured) + the gradient all_reduce
            out["exchange_bytes_per_rank_per_batch"] = learner.exchange_bytes_per_batch() + grad_bytes
            out["shard_records"] = {k: v for k, v in learner.shard_info.items() if k != "bytes_by_dest"}
        else:
            out["exchange_bytes_per_rank_per_batch"] = grad_bytes
    if stats:
        # after the timed region: one more batch with synchronised stage timers (the update's
        # stages on this rank: gather / learn (GAE + update; the learner rank's serial work under
        # "gather") / broadcast), then what that batch looked like to the update
        learner.exchange_timing = {}
        learner.collect()
        learner.update()
        learner.roll_over()
        torch.cuda.synchronize()
        st = dict(learner.exchange_timing)
        if dist:
            # every rank's stages (the same names on every rank under one exchange): the max over
            # ranks, as the batch waits for the slowest rank at each collective
            names = sorted(st)
            t = torch.tensor([st[k] for k in names], device=env.device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            st = dict(zip(names, t.tolist()))
            if exchange == "shard":
                # per-rank record traffic of the stats batch: bytes sent to other ranks and records
                world_ = dist.get_world_size()
                v = torch.zeros(3, world_, device=env.device, dtype=torch.float64)
                si = learner.shard_info
                v[:, dist.get_rank()] = torch.tensor([si.get("bytes_sent_to_other_ranks", 0),
                                                      si.get("actor_records_received", 0),
                                                      si.get("critic_records_received", 0)], dtype=torch.float64)
                dist.all_reduce(v, op=dist.ReduceOp.SUM)
                out["shard_bytes_sent_by_rank"] = [int(x) for x in v[0].tolist()]
                out["shard_records_received_by_rank"] = {"actor": [int(x) for x in v[1].tolist()],
                                                         "critic": [int(x) for x in v[2].tolist()]}
        out["update_stage_ms"] = st
        out["update_stage_ms_note"] = ("synchronised stage timers of one extra batch, max over ranks" if dist else
                                       "synchronised stage timers of one extra batch")
        learner.exchange_timing = None
        learner.collect()
        torch.cuda.synchronize()
        out["batch_stats"] = learner.batch_stats()
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) outside a torch.distributed.run environment: start N fresh rank
    processes through torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) with this
    script's own arguments, relay their output (rank 0 prints the JSON line) and return their
    exit code.  Runs before this process makes any GPU call; the ranks are children, never an
    exec of this process."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def check_faults(env):
    """A bounded hand-off wait that gave up leaves its envs' outputs invalid (fjsp_faults bit 0):
    a number measured over them is not reported."""
    w = env.faults()
    if w:
        raise SystemExit(f"bench: the step kernels reported fault word {w:#x} "
                         "(a hand-off wait gave up); no value reported")


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
    elif args.gpus is not None and args.gpus != int(env_world):
        sys.exit(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one GPU per rank; FJSP_BENCH_BACKEND=gloo rehearses the multi-rank logic with several
        # ranks on fewer GPUs (timing collectives only; stepping has no data-path collective)
        backend = os.environ.get("FJSP_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(local % torch.cuda.device_count())
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local % torch.cuda.device_count()))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    vec_env = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")

    N = args.envs
    base = rank * N
    env = vec_env.FJSPVecEnv(N, device=dev, env_id_base=base)
    if args.workload == "a2c":
        res = a2c_throughput(env, N, world, args.steps, args.warmup, args.batch_size, 25, dist,
                             dist.group.WORLD if dist else None, dedup=not args.no_dedup, exchange=args.exchange,
                             init=args.init)
        if rank == 0:
            out = {"metric": "env-steps/sec of the A2C training loop (BASELINE configs 4/5)",
                   "value": res["value"], "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
                   "warmup": args.warmup, "ms_per_step": res["ms_per_batch"], "higher_is_better": True,
                   "scaling": "weak", "vs_baseline": None, "dtype": "f32 (networks; k_policy: f32 operands as 3 bf16 planes on the MFMA, f32 accumulate) + int32/f64 (env)",
                   "data": "synthetic: envs seeded by global id, " + (
                       "random-init networks (torch.manual_seed(0))" if args.init == "random" else
                       "networks from the reference's trained checkpoints/model.pt"),
                   "config": {"workload": f"a2c_{N}envs", "envs_per_gpu": N, "global_envs": N * world,
                              "batch_size": args.batch_size, "num_orders": 25, "init": args.init,
                              "exchange": args.exchange if world > 1 else None,
                              "parallelism": f"env-shard x{world}" + (
                                  "" if world == 1 else ", experience gather into rank 0 + parameter broadcast"
                                  if args.exchange == "gather" else ", learner sharded by network: records "
                                  "all_to_all + one gradient all_reduce" if args.exchange == "shard"
                                  else ", one flat gradient all_reduce per batch")},
                   "a2c": res}
            print(json.dumps(out), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    env.reset(seeds=torch.arange(base, base + N), num_orders=args.num_orders)
    # the bench times its launches with its own events: the library's per-launch hipEvents
    # (fjsp_last_kernel_ms) would add two more event packets between launches (0.7 % of wall time
    # per 1 024-step launch, profiles/r04/ab_launch_gaps_lib_timing.json)
    nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
    nat.check(nat.lib().fjsp_set_option(env.handle, b"timing", 0))
    B = args.batch_steps                      # env-steps of every env per bench step
    chunk = max(1, min(args.chunk, args.steps * B))
    buf = vec_env.Buffers(chunk, N, dev, infos=False)
    stream = torch.cuda.current_stream(dev)

    def run(nsteps, step0, timing=None, chunk=chunk, buf=buf):
        done = 0
        while done < nsteps:
            k = min(chunk, nsteps - done)
            if timing is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            env.rollout(k, action_seed=1234, step0=step0 + done, masked=args.masked, buffers=buf)
            if timing is not None:
                e1.record(stream)
                timing.append((e0, e1, k))
            done += k
        return step0 + nsteps

    s0 = run(args.warmup * B, 0)
    kernel_name = env.last_kernel()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    timing = []
    t0 = time.perf_counter()
    run(args.steps * B, s0, timing)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    check_faults(env)
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = [a.elapsed_time(b) for a, b, _ in timing]
    kern_steps = [k for _, _, k in timing]
    full = [ms for ms, k in zip(kern_ms, kern_steps) if k == chunk] or kern_ms
    avg_launch_ms = float(np.mean(full))
    steps_per_launch = chunk
    total_env_steps = args.steps * B * N * world
    value = total_env_steps / elapsed
    achieved = ALGO_BYTES_FUSED * N * steps_per_launch / (avg_launch_ms * 1e-3) / 1e9
    # the same workload in 200-step launches (r01's first headline configuration), rank-local
    chunk_200 = None
    if chunk != 200 and args.steps * B >= 200 and not args.no_chunk_compare:
        buf200 = vec_env.Buffers(200, N, dev, infos=False)
        s1 = run(200, s0 + args.steps * B, chunk=200, buf=buf200)
        torch.cuda.synchronize()
        t200 = []
        tc = time.perf_counter()
        n200 = (args.steps * B // 200) * 200
        run(n200, s1, t200, chunk=200, buf=buf200)
        torch.cuda.synchronize()
        el200 = time.perf_counter() - tc
        ms200 = float(np.mean([a.elapsed_time(b) for a, b, _ in t200]))
        chunk_200 = {"value": n200 * N / el200, "unit": "env-steps/s", "steps_per_launch": 200,
                     "avg_launch_ms": ms200, "note": "rank-local, same workload in 200-step launches"}
        del buf200

    # one-launch-per-step mode (actions resident in HBM, k_step): the RL-loop path
    per_step = None
    if not args.no_step_mode:
        K = 200
        acts = torch.randint(0, 256, (K, 8, N), dtype=torch.int32, device=dev)
        nact = torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], dtype=torch.int32, device=dev).view(1, 8, 1)
        acts = ((acts * nact) >> 8).to(torch.uint8).contiguous()
        sbuf = vec_env.Buffers(1, N, dev, infos=False)
        for t in range(20):
            env.step(acts[t], buffers=sbuf)
        torch.cuda.synchronize()
        ev = []
        t1 = time.perf_counter()
        for t in range(K):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.step(acts[t], buffers=sbuf)
            e1.record(stream)
            ev.append((e0, e1))
        torch.cuda.synchronize()
        wall = time.perf_counter() - t1
        kms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        per_step = {"value": K * N / wall, "unit": "env-steps/s", "n_gpus": 1, "avg_kernel_ms": kms,
                    "kernel": env.last_kernel(), "algo_bytes_per_env_step": ALGO_BYTES_STEP,
                    "achieved_GBs": ALGO_BYTES_STEP * N / (kms * 1e-3) / 1e9,
                    "note": "one launch per step, actions u8[8][N] resident in HBM (rank 0)"}
        if rank == 0 and not args.no_dropin:
            try:
                per_step["host_actions"] = host_action_step(env, dev, N)
            except Exception as e:   # the headline metric does not depend on this leg
                per_step["host_actions"] = {"error": f"{type(e).__name__}: {e}"}
            ps = load_pmc(f"server_{N}envs")   # the resident server's HBM bytes (scripts/diag_server_pmc.py)
            if ps and ps.get("hbm_bytes_per_env_step") and "error" not in per_step["host_actions"]:
                per_step["host_actions"]["server_traffic_bytes_per_env_step"] = ps["hbm_bytes_per_env_step"]
                per_step["host_actions"]["server_traffic_source"] = f"profiles/pmc_server_{N}envs.json"

    # the reference-API path itself (FJSPParallelEnv.step with dict actions, one env)
    dropin = None
    if rank == 0 and world == 1 and not args.no_dropin:
        try:
            dropin = dropin_latency(dev)
        except Exception as e:   # the headline metric does not depend on this leg
            dropin = {"error": f"{type(e).__name__}: {e}"}

    # the same kernel at 16x the envs (65 536 on this GPU): how far the env-step approaches the
    # HBM roofline once occupancy allows (the headline stays the 4 096-env workload)
    scale = None
    if world == 1 and not args.no_scale:
        try:
            NS = 16 * N
            sch = min(chunk, 256)   # 32-bit output offsets: K x envs x 64 B < 4 GiB per launch
            senv = vec_env.FJSPVecEnv(NS, device=dev)
            senv.reset(seeds=torch.arange(NS), num_orders=args.num_orders)
            sbuf = vec_env.Buffers(sch, NS, dev, infos=False)
            senv.rollout(sch, action_seed=1234, masked=args.masked, buffers=sbuf)
            torch.cuda.synchronize()
            sms = []
            for r in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                senv.rollout(sch, action_seed=1234, step0=(r + 1) * sch, masked=args.masked, buffers=sbuf)
                e1.record(stream)
                torch.cuda.synchronize()
                sms.append(e0.elapsed_time(e1))
            sm = float(np.mean(sms))
            sach = ALGO_BYTES_FUSED * NS * sch / (sm * 1e-3) / 1e9
            scale = {"envs": NS, "value": NS * sch / (sm * 1e-3), "unit": "env-steps/s",
                     "avg_launch_ms": sm, "kernel": senv.last_kernel(), "achieved_GBs": sach,
                     "frac": sach / HBM_PEAK_GBS, "steps_per_launch": sch}
            del senv, sbuf
            torch.cuda.empty_cache()   # the 16x buffers (~15 GB) are not reused below
        except Exception as e:
            scale = {"error": f"{type(e).__name__}: {e}"}

    a2c = None
    if world == 1 and not args.no_a2c:
        try:
            aenv = vec_env.FJSPVecEnv(N, device=dev)
            # four warm-up batches: the first collect / update carry one-time costs (graph
            # capture, allocator growth, library kernel selection: ~0.3 s / ~0.9 s), and the
            # grouped update's tensor sizes change with every batch's distinct-input counts, so
            # the caching allocator needs a few batches to hold blocks for all of them
            a2c = a2c_throughput(aenv, N, 1, 6, 4, args.batch_size, 25, dedup=not args.no_dedup)
            del aenv
            aenv = vec_env.FJSPVecEnv(N, device=dev)
            # the same loop from the reference's trained checkpoint: the states a trained policy
            # visits set the grouped update's distinct-input counts and the forced-tile share
            a2c["trained_init"] = a2c_throughput(aenv, N, 1, 4, 4, args.batch_size, 25, dedup=not args.no_dedup,
                                                 init="trained")
            del aenv
            aenv = vec_env.FJSPVecEnv(N, device=dev)
            a2c["dense_update"] = a2c_throughput(aenv, N, 1, 3, 2, args.batch_size, 25, dedup=False, stats=False)
            del aenv
        except Exception as e:   # the headline metric does not depend on this leg
            a2c = {"error": f"{type(e).__name__}: {e}"}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args)

    workload = f"fjsp_step_{N}envs"
    # HBM bytes from the PMC passes (profiles/pmc_<workload>.json, scripts/gpu_pmc.sh): keyed per
    # env-step so the figure applies to this launch length (exact when the profiled launch length
    # is this one, else scaled; traffic_source says which)
    pmc = load_pmc(workload)
    traffic, traffic_src = None, None
    if pmc and pmc.get("envs") == N and pmc.get("kernel_variant") == kernel_name and pmc.get("hbm_bytes_per_env_step"):
        traffic = pmc["hbm_bytes_per_env_step"] * N * steps_per_launch
        traffic_src = (f"profiles/pmc_{workload}.json, {pmc.get('steps_per_launch')}-step launches"
                       + ("" if pmc.get("steps_per_launch") == steps_per_launch else ", scaled per env-step"))
    if per_step is not None:
        pk = load_pmc(f"k_step_{N}envs")
        if pk and pk.get("kernel_variant") == per_step["kernel"] and pk.get("hbm_bytes_per_env_step"):
            per_step["traffic_bytes_per_env_step"] = pk["hbm_bytes_per_env_step"]
            per_step["traffic_source"] = f"profiles/pmc_k_step_{N}envs.json"
    if rank == 0:
        out = {
            "metric": "env-steps/sec (all agents) at N parallel envs, 1/2/4/8 MI355X",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32+f64",
            "data": "synthetic: random actions from the on-device counter RNG, envs seeded by global id",
            "config": {"workload": workload, "envs_per_gpu": N, "global_envs": N * world,
                       "num_orders": args.num_orders, "policy": "masked-random" if args.masked else "random",
                       "steps_per_launch": steps_per_launch, "kernel": kernel_name,
                       "bench_step": f"one rollout batch = {B} env-steps of each of the {N} envs",
                       "env_steps_per_bench_step": B * N * world,
                       "parallelism": f"env-shard x{world} (no data-path collective)"},
            "agent_steps_per_s": value * 8,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel_name, "avg_launch_ms": avg_launch_ms,
                         "algo_bytes_per_env_step": ALGO_BYTES_FUSED,
                         # SURVEY.md 8(d) prices an env-step at 219 B, 8 of them the u8 actions
                         # read from HBM; this kernel draws its actions on the device, so its
                         # algorithmic bytes are the 211 B of outputs (the 219 B figures beside)
                         "achieved_219B": achieved * ALGO_BYTES_STEP / ALGO_BYTES_FUSED,
                         "frac_219B": achieved * ALGO_BYTES_STEP / ALGO_BYTES_FUSED / HBM_PEAK_GBS,
                         "env_steps_per_launch": N * steps_per_launch},
            "cpu_baseline": cpu,
            "chunk_200": chunk_200,
            "per_step_launch": per_step,
            "dropin_n1_us_per_step": dropin.get("dropin_n1_us_per_step") if dropin else None,
            "dropin": dropin,
            "a2c_training": a2c,
            "scale_16x_envs": scale,
            "state_bytes_per_env": env.state_bytes_per_env(),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
