"""Host cost of engine.step_plan vs the GPU time of one step graph (cfg3 fp32): is the GPU idle
between graph replays because of the host?"""
import sys
import time
import torch
sys.path.insert(0, '.')
import bench  # noqa: E402

dev = torch.device('cuda:0')
cfg = sys.argv[1] if len(sys.argv) > 1 else 'cfg3'
w = bench.CONFIGS[cfg](dev, 0, True, bf16=len(sys.argv) > 2)
for _ in range(20):
    w.step()
torch.cuda.synchronize()
N = 300
t0 = time.perf_counter()
for _ in range(N):
    w.step()
th = time.perf_counter() - t0
torch.cuda.synchronize()
tt = time.perf_counter() - t0
print('step_plan: host %.1f us/step, total %.1f us/step' % (th / N * 1e6, tt / N * 1e6))
g = next(iter(w.eng._graphs.values()))[0]
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    g.replay()
th = time.perf_counter() - t0
torch.cuda.synchronize()
tt = time.perf_counter() - t0
print('bare replay: host %.1f us/step, total %.1f us/step' % (th / N * 1e6, tt / N * 1e6))
