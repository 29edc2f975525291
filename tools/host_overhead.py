"""Host-side cost of one eager log_prob call (tiny batch: GPU time negligible)."""
import sys, time, cProfile, pstats
sys.path.insert(0, "normalizing-flows-study_amd"); sys.path.insert(0, ".")
import torch
import bench

dev = torch.device("cuda:0")
m, d, _, _, _ = bench.build("cfg2")
m = m.to(dev).eval()
flow = m.flow
x = torch.randn(1024, d, device=dev)
with torch.no_grad():
    for _ in range(20):
        flow.log_prob(x, return_sums=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        flow.log_prob(x, return_sums=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
print(f"host issue {1e6 * (t1 - t0) / 200:.1f} us/call, wall {1e6 * (t2 - t0) / 200:.1f} us/call")
pr = cProfile.Profile()
with torch.no_grad():
    pr.enable()
    for _ in range(200):
        flow.log_prob(x, return_sums=True)
    pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
