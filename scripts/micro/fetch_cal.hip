// FETCH_SIZE / WRITE_SIZE calibration per access width (VERDICT r3 "make traffic trustworthy").
//
// MI355X_MICROARCH.md section HBM calibrates the gfx950 FETCH_SIZE correction (x2) only for
// 16-byte-per-lane streaming reads.  The kernels of libmep_hip.so also read with dword loads
// (k_wgrad: 32 lanes = 128 contiguous bytes per half-wave, two rows per wave-instruction), 8-byte
// loads, LDS-DMA (buffer_load ... lds, 4 and 16 bytes per lane), sub-line row slices (attention:
// 64 bytes of a 384 / 512-byte row per head) and 2-byte loads (bf16 storage).  Each kernel here
// touches a KNOWN number of bytes of a 1 GiB buffer (far past the 256 MiB Infinity Cache) exactly
// once per dispatch; rocprofv3 --pmc passes over this program give counter bytes / known bytes
// per access width (scripts/fetch_cal.py writes the table, bench.py applies it per kernel).
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro/fetch_cal scripts/micro/fetch_cal.hip
//   ./scripts/micro/fetch_cal        -> one JSON line per kernel: {"kernel", "bytes", "us"}
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int TPB = 256;
constexpr int NWG = 2048;   // 8 workgroups per CU, grid-stride

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// -- contiguous reads: every wave-instruction reads 64 x W contiguous bytes
template <int W>
__global__ __launch_bounds__(TPB) void k_rd(const char* __restrict__ src, size_t n_bytes, float* __restrict__ out) {
    const size_t per_instr = 64 * W;
    const size_t n_instr = n_bytes / per_instr;
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const size_t nwaves = (size_t)gridDim.x * (TPB / 64);
    float acc = 0.f;
    for (size_t i = wave; i < n_instr; i += nwaves) {
        const char* p = src + i * per_instr + (size_t)lane * W;
        if (W == 2) acc += (float)*reinterpret_cast<const unsigned short*>(p);
        if (W == 4) acc += *reinterpret_cast<const float*>(p);
        if (W == 8) { const f32x2 v = *reinterpret_cast<const f32x2*>(p); acc += v[0] + v[1]; }
        if (W == 16) { const f32x4 v = *reinterpret_cast<const f32x4*>(p); acc += v[0] + v[1] + v[2] + v[3]; }
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;   // keeps the loads; never true on the zeroed buffer
}

// -- k_wgrad's shape: dword loads, lanes 0-31 read 128 contiguous bytes of one row and lanes 32-63
// 128 bytes of the next row (row stride RS bytes); every byte of every row read once
template <int RS>
__global__ __launch_bounds__(TPB) void k_rd_seg128(const char* __restrict__ src, size_t n_bytes, float* __restrict__ out) {
    constexpr int SEGS = RS / 128;                 // 128-byte segments per row
    const size_t n_rows = n_bytes / RS;
    const size_t n_instr = n_rows / 2 * SEGS;      // row pairs x segments
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const size_t nwaves = (size_t)gridDim.x * (TPB / 64);
    float acc = 0.f;
    for (size_t i = wave; i < n_instr; i += nwaves) {
        const size_t pair = i / SEGS, seg = i % SEGS;
        const char* p = src + (2 * pair + (lane >> 5)) * RS + seg * 128 + 4 * (lane & 31);
        acc += *reinterpret_cast<const float*>(p);
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

// -- the attention's shape: 16 rows per wave-instruction, 4 lanes x 16 bytes = the 64-byte head
// slice of each row; rows of RS bytes; only the first 64 bytes of each row are read (the known
// byte count is 64 per row: anything above is over-fetch of the partial line)
template <int RS, int SLICE>
__global__ __launch_bounds__(TPB) void k_rd_slice(const char* __restrict__ src, size_t n_bytes, float* __restrict__ out) {
    constexpr int LPR = SLICE / 16;                // lanes per row
    constexpr int RPI = 64 / LPR;                  // rows per wave-instruction
    const size_t n_rows = n_bytes / RS;
    const size_t n_instr = n_rows / RPI;
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const size_t nwaves = (size_t)gridDim.x * (TPB / 64);
    float acc = 0.f;
    for (size_t i = wave; i < n_instr; i += nwaves) {
        const char* p = src + (i * RPI + lane / LPR) * RS + 16 * (lane % LPR);
        const f32x4 v = *reinterpret_cast<const f32x4*>(p);
        acc += v[0] + v[1] + v[2] + v[3];
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

// -- LDS-DMA (buffer_load ... lds): W = 4 or 16 bytes per lane, 64 x W contiguous bytes per
// wave-instruction, into a per-wave LDS slot (contents unused)
template <int W>
__global__ __launch_bounds__(TPB) void k_lds_dma(const char* __restrict__ src, size_t n_bytes, float* __restrict__ out) {
    __shared__ float slot[TPB / 64][64 * W / 4];
    typedef __attribute__((address_space(3))) void lvoid;
    const size_t per_instr = 64 * W;
    const size_t n_instr = n_bytes / per_instr;
    const size_t wave = (size_t)__builtin_amdgcn_readfirstlane(blockIdx.x * (TPB / 64) + (threadIdx.x >> 6));
    const size_t nwaves = (size_t)gridDim.x * (TPB / 64);
    const int lane = threadIdx.x & 63;
    for (size_t i = wave; i < n_instr; i += nwaves) {
        // one descriptor per 1 GiB window is enough: offsets stay below 2^31
        const char* base = src + i * per_instr;
        const __amdgpu_buffer_rsrc_t rs = rsrc(base, (uint32_t)per_instr);
        if constexpr (W == 4) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lvoid*)&slot[threadIdx.x >> 6][0], 4, lane * 4, 0, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lvoid*)&slot[threadIdx.x >> 6][0], 16, lane * 16, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (slot[0][threadIdx.x & 63] == 1.2345f) out[blockIdx.x] = 1.f;
}

// -- stores: W bytes per lane, 64 x W contiguous bytes per wave-instruction
template <int W>
__global__ __launch_bounds__(TPB) void k_wr(char* __restrict__ dst, size_t n_bytes) {
    const size_t per_instr = 64 * W;
    const size_t n_instr = n_bytes / per_instr;
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const size_t nwaves = (size_t)gridDim.x * (TPB / 64);
    for (size_t i = wave; i < n_instr; i += nwaves) {
        char* p = dst + i * per_instr + (size_t)lane * W;
        if (W == 2) *reinterpret_cast<unsigned short*>(p) = (unsigned short)lane;
        if (W == 4) *reinterpret_cast<float*>(p) = (float)lane;
        if (W == 16) *reinterpret_cast<f32x4*>(p) = f32x4{1.f, 2.f, 3.f, (float)lane};
    }
}

// -- k_wgrad's stores / the epilogues' row stores at 64 bytes per row: 16 rows x 64 bytes
template <int RS>
__global__ __launch_bounds__(TPB) void k_wr_slice64(char* __restrict__ dst, size_t n_bytes) {
    const size_t n_rows = n_bytes / RS;
    const size_t n_instr = n_rows / 16;
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const size_t nwaves = (size_t)gridDim.x * (TPB / 64);
    for (size_t i = wave; i < n_instr; i += nwaves) {
        char* p = dst + (i * 16 + lane / 4) * RS + 16 * (lane % 4);
        *reinterpret_cast<f32x4*>(p) = f32x4{1.f, 2.f, 3.f, (float)lane};
    }
}

int main() {
    const size_t N = (size_t)1 << 30;   // 1 GiB, past the 256 MiB Infinity Cache
    char *src, *dst;
    float* out;
    CHECK(hipMalloc(&src, N));
    CHECK(hipMalloc(&dst, N));
    CHECK(hipMalloc(&out, NWG * sizeof(float)));
    CHECK(hipMemset(src, 0, N));
    CHECK(hipMemset(dst, 0, N));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 3;
    auto run = [&](const char* name, double bytes, auto launch) -> int {
        launch();   // warm
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"us\": %.2f, \"TBps\": %.3f}\n", name, bytes, 1e3 * ms / reps,
               bytes / (1e-3 * ms / reps) / 1e12);
        fflush(stdout);
        return 0;
    };
    const dim3 g(NWG), b(TPB);
    int rc = 0;
    rc |= run("k_rd<2>", (double)N, [&] { k_rd<2><<<g, b>>>(src, N, out); });
    rc |= run("k_rd<4>", (double)N, [&] { k_rd<4><<<g, b>>>(src, N, out); });
    rc |= run("k_rd<8>", (double)N, [&] { k_rd<8><<<g, b>>>(src, N, out); });
    rc |= run("k_rd<16>", (double)N, [&] { k_rd<16><<<g, b>>>(src, N, out); });
    rc |= run("k_rd_seg128<384>", (double)(N / 768 * 768), [&] { k_rd_seg128<384><<<g, b>>>(src, N, out); });
    rc |= run("k_rd_seg128<512>", (double)N, [&] { k_rd_seg128<512><<<g, b>>>(src, N, out); });
    // slices: known bytes = SLICE per row read
    rc |= run("k_rd_slice<384,64>", (double)(N / 384 / 16 * 16) * 64, [&] { k_rd_slice<384, 64><<<g, b>>>(src, N, out); });
    rc |= run("k_rd_slice<512,64>", (double)(N / 512 / 16 * 16) * 64, [&] { k_rd_slice<512, 64><<<g, b>>>(src, N, out); });
    rc |= run("k_rd_slice<512,128>", (double)(N / 512 / 8 * 8) * 128, [&] { k_rd_slice<512, 128><<<g, b>>>(src, N, out); });
    rc |= run("k_lds_dma<4>", (double)N, [&] { k_lds_dma<4><<<g, b>>>(src, N, out); });
    rc |= run("k_lds_dma<16>", (double)N, [&] { k_lds_dma<16><<<g, b>>>(src, N, out); });
    rc |= run("k_wr<2>", (double)N, [&] { k_wr<2><<<g, b>>>(dst, N); });
    rc |= run("k_wr<4>", (double)N, [&] { k_wr<4><<<g, b>>>(dst, N); });
    rc |= run("k_wr<16>", (double)N, [&] { k_wr<16><<<g, b>>>(dst, N); });
    rc |= run("k_wr_slice64<384>", (double)(N / 384 / 16 * 16) * 64, [&] { k_wr_slice64<384><<<g, b>>>(dst, N); });
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    CHECK(hipFree(out));
    return rc;
}
