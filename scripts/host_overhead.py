"""Host-side cost of one bench step (graph replay path): wall time of K step() calls without a
device sync vs with one, plus a cProfile of the host code (development aid)."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mep_import  # noqa: E402

mep_import.load()


def main():
    import bench
    dev = torch.device('cuda:0')
    bf16 = len(sys.argv) > 1 and sys.argv[1] == 'bf16'
    work = bench.Cfg3(dev, 0, graph=True, bf16=bf16)
    for _ in range(20):
        work.step()
    torch.cuda.synchronize()
    K = 300
    t0 = time.perf_counter()
    for _ in range(K):
        work.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print('host issue %.1f us/step, wall %.1f us/step' % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(K):
        work.step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats('cumulative').print_stats(18)


if __name__ == '__main__':
    main()
