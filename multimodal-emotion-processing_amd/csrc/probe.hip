// mep_hbm_probe: the measured HBM peak bench.py reports beside the 8 TB/s spec (SURVEY.md 8(d):
// "vendor spec AND a measured copy-kernel peak on the box").  Not on the training path.
//
// Grid-stride streaming over n16 16-byte units with UNROLL independent dwordx4 accesses in flight
// per thread, 256-thread workgroups, 8 per CU.  Adjacent lanes touch adjacent 16-byte units, so a
// wave instruction covers 1 KiB of contiguous memory (8 whole 128-byte lines).
//   mode 0 (copy): dst[i] = src[i]            -> 2 * 16 * n16 bytes
//   mode 1 (read): every unit loaded, one dword per thread written (the xor of what it read, so
//                  the loads cannot be dropped) -> 16 * n16 bytes (+ 4 per thread)
//   mode 2 (write): dst[i] = 0                -> 16 * n16 bytes
// mep_stamp: a one-wave kernel storing the real-time counter, the bench's in-step launch timer.
#include "common.h"

namespace {

using namespace mep;

constexpr int PROBE_THREADS = 256;
constexpr int PROBE_UNROLL = 8;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef MEP_G u32x4 gu32x4;

template <int MODE>
__global__ __launch_bounds__(PROBE_THREADS) void k_hbm_probe(uint64_t src_p, uint64_t dst_p, int64_t n16) {
    const gu32x4* __restrict__ src = G<const u32x4>(src_p);
    gu32x4* __restrict__ dst = G<u32x4>(dst_p);
    const int64_t nth = (int64_t)gridDim.x * PROBE_THREADS;
    const int64_t tid = (int64_t)blockIdx.x * PROBE_THREADS + threadIdx.x;
    u32x4 acc = u32x4{0u, 0u, 0u, 0u};
    int64_t i = tid;
    // main loop: PROBE_UNROLL accesses per thread in flight, all in range
    for (; i + (PROBE_UNROLL - 1) * nth < n16; i += PROBE_UNROLL * nth) {
        if (MODE == 2) {
#pragma unroll
            for (int u = 0; u < PROBE_UNROLL; ++u) dst[i + u * nth] = u32x4{0u, 0u, 0u, 0u};
        } else {
            u32x4 v[PROBE_UNROLL];
#pragma unroll
            for (int u = 0; u < PROBE_UNROLL; ++u) v[u] = src[i + u * nth];
            if (MODE == 0) {
#pragma unroll
                for (int u = 0; u < PROBE_UNROLL; ++u) dst[i + u * nth] = v[u];
            } else {
#pragma unroll
                for (int u = 0; u < PROBE_UNROLL; ++u) acc ^= v[u];
            }
        }
    }
    for (; i < n16; i += nth) {
        if (MODE == 2) dst[i] = u32x4{0u, 0u, 0u, 0u};
        else if (MODE == 0) dst[i] = src[i];
        else acc ^= src[i];
    }
    if (MODE == 1) {
        MEP_G unsigned* o = reinterpret_cast<MEP_G unsigned*>(dst);
        o[tid] = acc.x ^ acc.y ^ acc.z ^ acc.w;
    }
}

// The blocked variant: workgroup w streams its own contiguous span of the buffer, 32 KiB per step
// (8 unrolled 1-KiB wave instructions of 256 threads), so consecutive requests of a CU stay in one
// DRAM page run; NT: nontemporal (streaming) loads and stores.
template <int MODE, bool NT>
__global__ __launch_bounds__(PROBE_THREADS) void k_hbm_probe_blk(uint64_t src_p, uint64_t dst_p, int64_t n16) {
    const gu32x4* __restrict__ src = G<const u32x4>(src_p);
    gu32x4* __restrict__ dst = G<u32x4>(dst_p);
    constexpr int64_t STEP = (int64_t)PROBE_THREADS * PROBE_UNROLL;
    const int64_t per = ((n16 + gridDim.x - 1) / gridDim.x + STEP - 1) / STEP * STEP;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = min(lo + per, n16);
    u32x4 acc = u32x4{0u, 0u, 0u, 0u};
    int64_t i = lo + threadIdx.x;
    for (; i + (PROBE_UNROLL - 1) * PROBE_THREADS < hi; i += STEP) {
        if (MODE == 2) {
#pragma unroll
            for (int u = 0; u < PROBE_UNROLL; ++u) {
                if (NT) __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, &dst[i + u * PROBE_THREADS]);
                else dst[i + u * PROBE_THREADS] = u32x4{0u, 0u, 0u, 0u};
            }
        } else {
            u32x4 v[PROBE_UNROLL];
#pragma unroll
            for (int u = 0; u < PROBE_UNROLL; ++u)
                v[u] = NT ? __builtin_nontemporal_load(&src[i + u * PROBE_THREADS]) : src[i + u * PROBE_THREADS];
            if (MODE == 0) {
#pragma unroll
                for (int u = 0; u < PROBE_UNROLL; ++u) {
                    if (NT) __builtin_nontemporal_store(v[u], &dst[i + u * PROBE_THREADS]);
                    else dst[i + u * PROBE_THREADS] = v[u];
                }
            } else {
#pragma unroll
                for (int u = 0; u < PROBE_UNROLL; ++u) acc ^= v[u];
            }
        }
    }
    for (; i < hi; i += PROBE_THREADS) {
        if (MODE == 2) dst[i] = u32x4{0u, 0u, 0u, 0u};
        else if (MODE == 0) dst[i] = src[i];
        else acc ^= src[i];
    }
    if (MODE == 1) {
        MEP_G unsigned* o = reinterpret_cast<MEP_G unsigned*>(dst);
        o[(int64_t)blockIdx.x * PROBE_THREADS + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
    }
}

// one lane writes the 100-MHz real-time counter (s_memrealtime) when the kernel starts: placed
// between the launches of a captured step, consecutive stamps bracket each launch's device time
__global__ __launch_bounds__(64) void k_stamp(uint64_t out) {
    if (threadIdx.x == 0) *G<unsigned long long>(out) = wall_clock64();
}

}  // namespace

extern "C" int mep_hbm_probe(const void* src, void* dst, int64_t n16, int mode_flags, int n_wg, mep_stream_t stream) {
    const int mode = mode_flags & 3;
    const bool blocked = mode_flags & MEP_PROBE_BLOCKED, nt = mode_flags & MEP_PROBE_NT;
    if (n16 <= 0 || mode > 2 || (mode_flags & ~(3 | MEP_PROBE_BLOCKED | MEP_PROBE_NT)) || n_wg <= 0 || (mode != 2 && !src) || !dst ||
        (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15)) {
        mep_set_error("mep_hbm_probe: bad arguments (16-byte aligned buffers, n16 > 0, mode 0..2, n_wg > 0)");
        return -1;
    }
    const uint64_t s = reinterpret_cast<uint64_t>(src), d = reinterpret_cast<uint64_t>(dst);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (blocked) {
#define MEP_PB(M) do { if (nt) hipLaunchKernelGGL((k_hbm_probe_blk<M, true>), dim3(n_wg), dim3(PROBE_THREADS), 0, st, s, d, n16); \
                       else hipLaunchKernelGGL((k_hbm_probe_blk<M, false>), dim3(n_wg), dim3(PROBE_THREADS), 0, st, s, d, n16); } while (0)
        if (mode == 0) MEP_PB(0); else if (mode == 1) MEP_PB(1); else MEP_PB(2);
#undef MEP_PB
        return mep_check_launch("mep_hbm_probe");
    }
    if (mode == 0) hipLaunchKernelGGL(k_hbm_probe<0>, dim3(n_wg), dim3(PROBE_THREADS), 0, st, s, d, n16);
    else if (mode == 1) hipLaunchKernelGGL(k_hbm_probe<1>, dim3(n_wg), dim3(PROBE_THREADS), 0, st, s, d, n16);
    else hipLaunchKernelGGL(k_hbm_probe<2>, dim3(n_wg), dim3(PROBE_THREADS), 0, st, s, d, n16);
    return mep_check_launch("mep_hbm_probe");
}

extern "C" int mep_stamp(void* slots, int i, mep_stream_t stream) {
    if (!slots || i < 0 || (reinterpret_cast<uintptr_t>(slots) & 7)) {
        mep_set_error("mep_stamp: bad arguments (8-byte aligned slots, i >= 0)");
        return -1;
    }
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
               reinterpret_cast<uint64_t>(slots) + 8ull * (uint64_t)i);
    return mep_check_launch("mep_stamp");
}

extern "C" int mep_stamp_khz(void) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) {
        mep_set_error("mep_stamp_khz: hipDeviceGetAttribute(hipDeviceAttributeWallClockRate) failed");
        return -1;
    }
    return khz;
}
