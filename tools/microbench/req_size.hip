// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/req_size tools/microbench/req_size.hip
// Calibration of the L2 -> fabric read-request counters (TCC_EA0_RDREQ, TCC_BUBBLE, TCC_EA0_RDREQ_32B, FETCH_SIZE)
// on gfx950 for the access patterns k_scan_ax issues (MI355X_MICROARCH.md §HBM: "calibrate on a known byte count in
// your own access pattern"). Each kernel moves a known number of distinct bytes from a buffer far larger than the
// 256 MiB Infinity Cache (no reuse), so bytes per request = known bytes / requests:
//   k_stream16  every lane loads 16 B, consecutive lanes consecutive 16 B (the staging stream of k_scan_ax)
//   k_gather16  every lane loads 16 B of its own random 128-B line (the run-granule / bucket-word loads)
//   k_gather64  every lane loads 4 x 16 B = one random 64-B bucket (the anchor-bucket loads)
//   k_gather128 every lane loads 8 x 16 B = one random 128-B line
// Usage: req_size [MiB]   prints one JSON line per kernel: distinct bytes, best-of-5 ms (HIP events).
// Run under rocprofv3 --pmc to read the counters per kernel (scripts/calibrate_counters.sh).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ void k_stream16(const uint4* __restrict__ s, uint64_t n16, unsigned* out) {
    unsigned acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 a = s[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// line index of gather i: a bijection of [0, n_lines) (odd multiplier mod a power of two), so no line is read twice
__device__ __forceinline__ uint64_t line_of(uint64_t i, uint64_t n_lines) {
    return (i * 0x9E3779B97F4A7C15ull) & (n_lines - 1);
}

template <int PARTS>  // 16-B parts per gather: 1, 4 (64 B) or 8 (128 B)
__global__ void k_gather(const uint4* __restrict__ s, uint64_t n_lines, uint64_t n_gathers, unsigned* out) {
    unsigned acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_gathers;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4* p = s + line_of(i, n_lines) * 8;  // 128-B line
#pragma unroll
        for (int t = 0; t < PARTS; ++t) {
            const uint4 a = p[t];
            acc ^= a.x ^ a.y ^ a.z ^ a.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2048;  // power of two
    const uint64_t bytes = mib << 20, n_lines = bytes / 128;
    uint4* buf = nullptr;
    unsigned* out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 0x5A, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double distinct, auto launch) {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best) best = ms;
        }
        std::printf("{\"kernel\": \"%s\", \"distinct_bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", name, distinct,
                    best, distinct / best / 1e6);
        std::fflush(stdout);
    };
    const uint64_t quarter = n_lines / 4;  // gathers touch a quarter of the lines: distinct, spread over the buffer
    timeit("k_stream16", (double)bytes, [&] {
        hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, buf, bytes / 16, out);
    });
    timeit("k_gather16", 16.0 * quarter, [&] {
        hipLaunchKernelGGL(k_gather<1>, dim3(8192), dim3(256), 0, 0, buf, n_lines, quarter, out);
    });
    timeit("k_gather64", 64.0 * quarter, [&] {
        hipLaunchKernelGGL(k_gather<4>, dim3(8192), dim3(256), 0, 0, buf, n_lines, quarter, out);
    });
    timeit("k_gather128", 128.0 * quarter, [&] {
        hipLaunchKernelGGL(k_gather<8>, dim3(8192), dim3(256), 0, 0, buf, n_lines, quarter, out);
    });
    CK(hipGetLastError());
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
