import sys, os, time, importlib, torch
sys.path.insert(0, "/root/repo")
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
N = 4096
env = ve.FJSPVecEnv(N)
L = A.VecMultiAgentA2C(env, batch_size=256, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
for b in range(5):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    L.collect(); torch.cuda.synchronize(); t1 = time.perf_counter()
    ret, adv = L.advantages(); torch.cuda.synchronize(); t2 = time.perf_counter()
    L.update(ret, adv); torch.cuda.synchronize(); t3 = time.perf_counter()
    L.roll_over()
    print(b, "collect %.1f adv %.1f update %.1f ms" % ((t1-t0)*1e3, (t2-t1)*1e3, (t3-t2)*1e3), flush=True)
