"""Isolated check of the mechanism behind r04's graph-captured-update divergence:
two hipGraphs captured into ONE shared memory pool, A then B.  A's intermediate is freed when its
capture ends, so B's capture may place its OUTPUT in that memory; replaying A again (out of
capture order, as the removed update's least-recently-used replay did) then writes A's
intermediate over B's live output.  The same graphs in private pools, and the shared pool replayed
in capture order, keep B's output.  Prints JSON."""
import json

import torch

n = 1 << 22
x = torch.arange(n, device="cuda", dtype=torch.float32)


def run(shared, out_of_order):
    pool = torch.cuda.graph_pool_handle() if shared else None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):                      # warm-up off the capture, per the capture rules
        for _ in range(2):
            (x * 2 + 1).sum()
    torch.cuda.current_stream().wait_stream(s)
    gA, gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gA, pool=pool):
        t = x * 2.0                                 # A's intermediate (freed after the capture)
        a_out = t + 1.0
        t_ptr = t.data_ptr()
        del t
    with torch.cuda.graph(gB, pool=pool if shared else None):
        b_out = x * 3.0                             # B's output, kept alive by this reference
    gA.replay()
    gB.replay()
    if out_of_order:
        gA.replay()                                 # A after B: not capture order
    torch.cuda.synchronize()
    ok = bool(torch.equal(b_out, x * 3.0)) and bool(torch.equal(a_out, x * 2.0 + 1.0))
    return {"shared_pool": shared, "replay_out_of_capture_order": out_of_order,
            "b_output_aliases_a_intermediate": b_out.data_ptr() == t_ptr, "outputs_correct": ok}


print(json.dumps([run(True, True), run(True, False), run(False, True)]))
