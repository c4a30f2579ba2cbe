"""Do independent branches of a captured hipGraph run concurrently?  Two torch.cuda._sleep
kernels (one workgroup each) on a forked side stream vs the same two on one stream, eager and
captured; prints the per-replay times."""
import time

import torch


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    cyc = 2_000_000
    side = torch.cuda.Stream()

    def serial():
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)

    def forked():
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        main_s.wait_stream(side)

    print('eager serial %.0f us, forked %.0f us' % (timeit(serial), timeit(forked)))
    for name, fn in (('serial', serial), ('forked', forked)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fn()
        print('graph %s %.0f us' % (name, timeit(g.replay)))


if __name__ == '__main__':
    main()
