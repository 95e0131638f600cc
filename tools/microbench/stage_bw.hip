// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/stage_bw tools/microbench/stage_bw.hip (results: profiles/r02/stage_bw.jsonl)
// Microbenchmark (GPU box): read rate of the read-staging access pattern of k_scan_ax, isolated from the kernel.
// Reads of 150 bases laid end to end (seq + qual buffers, 1 M reads by default). Variants:
//   0 grid-stride 16-B loads over the whole buffers (the torch-like sweep)
//   1 one wave per group of 64 reads (the group's byte range, 16 B per lane per instruction), one group per wave
//   2 as 1, but a fixed grid of 1024 blocks dealing groups round robin
//   3 as 1, with 128 VGPRs pinned by a dummy register array (the scan kernel's occupancy: 4 waves per SIMD)
// Usage: stage_bw [reads]   prints one JSON line per variant (best of 10 launches, HIP events)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ void k_sweep(const uint4* __restrict__ s, const uint4* __restrict__ q, uint64_t n16, unsigned* out) {
    unsigned acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 a = s[i], b = q[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <bool PIN>
__global__ __launch_bounds__(256, 4) void k_groups(const uint8_t* __restrict__ s, const uint8_t* __restrict__ q,
                                                  const uint64_t* __restrict__ off, uint64_t n_reads, unsigned* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * 4, gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t ng = (n_reads + 63) / 64;
    unsigned acc = 0;
    unsigned pin[PIN ? 96 : 1];
    if (PIN)
        for (int i = 0; i < (PIN ? 96 : 1); ++i) pin[i] = __builtin_amdgcn_readfirstlane(i * lane);
    for (uint64_t g = gw; g < ng; g += nw) {
        const uint64_t r0 = g * 64, r1 = r0 + 64 < n_reads ? r0 + 64 : n_reads;
        const uint64_t a = off[r0] & ~15ull, e = off[r1];
        for (uint64_t p = a + 16 * lane; p < e; p += 1024) {
            const uint4 x = *reinterpret_cast<const uint4*>(s + p), y = *reinterpret_cast<const uint4*>(q + p);
            acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w;
        }
    }
    if (PIN)
        for (int i = 0; i < (PIN ? 96 : 1); ++i) acc += pin[i];
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
    const uint64_t L = 150, bytes = n * L;
    std::vector<uint64_t> off(n + 1);
    for (uint64_t i = 0; i <= n; ++i) off[i] = i * L;
    uint8_t *s, *q;
    uint64_t* d_off;
    unsigned* out;
    CK(hipMalloc(&s, bytes + 64));
    CK(hipMalloc(&q, bytes + 64));
    CK(hipMalloc(&d_off, (n + 1) * 8));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(s, 'A', bytes + 64));
    CK(hipMemset(q, 'I', bytes + 64));
    CK(hipMemcpy(d_off, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t groups = (n + 63) / 64;
    for (int v = 0; v < 4; ++v) {
        float best = 1e9f;
        for (int it = 0; it < 11; ++it) {
            CK(hipEventRecord(e0));
            if (v == 0)
                hipLaunchKernelGGL(k_sweep, dim3(4096), dim3(256), 0, 0, (const uint4*)s, (const uint4*)q, bytes / 16, out);
            else if (v == 1)
                hipLaunchKernelGGL(k_groups<false>, dim3((groups + 3) / 4), dim3(256), 0, 0, s, q, d_off, n, out);
            else if (v == 2)
                hipLaunchKernelGGL(k_groups<false>, dim3(1024), dim3(256), 0, 0, s, q, d_off, n, out);
            else
                hipLaunchKernelGGL(k_groups<true>, dim3((groups + 3) / 4), dim3(256), 0, 0, s, q, d_off, n, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0 && ms < best) best = ms;
        }
        std::printf("{\"variant\": %d, \"reads\": %llu, \"ms\": %.4f, \"GBps\": %.1f}\n", v, (unsigned long long)n, best,
                    2.0 * bytes / best / 1e6);
    }
    return 0;
}
