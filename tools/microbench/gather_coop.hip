// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/gather_coop tools/microbench/gather_coop.hip
// How fast do dependent chains of random 64-B bucket reads run when every lane reads its own bucket with four 16-B
// loads (k_scan_ax's anchor lookups: 4 wave-instructions, each touching 64 lines) against four lanes sharing one
// bucket (each wave-instruction touches 16 lines, 64 contiguous bytes each; the owner lane gets the bucket's digest
// back through cross-lane moves)? Persistent grid of 5 x 256-thread blocks per CU, every lane runs one chain of
// `iters` dependent lookups (the next bucket index comes from the bucket just read).
// Usage: gather_coop [table MiB] [iters]   prints one JSON line per pattern: ms (best of 5), G lookups/s.
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

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

// pattern A: one lane, one bucket, four 16-B loads
__global__ void k_lane64(const uint4* __restrict__ t, uint32_t nb, uint32_t iters, unsigned* out) {
    uint32_t s = mix(blockIdx.x * blockDim.x + threadIdx.x + 1u);
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t b = (uint32_t)(((uint64_t)s * nb) >> 32);
        const uint4 a0 = t[4ull * b], a1 = t[4ull * b + 1], a2 = t[4ull * b + 2], a3 = t[4ull * b + 3];
        s = mix(s ^ a0.x ^ a1.y ^ a2.z ^ a3.w ^ a0.w);
    }
    if (s == 0x12345678u) out[0] = s;
}

// pattern B: four lanes share one bucket. Instruction i serves the chains of lanes 16 i .. 16 i + 15: lane l loads
// part l % 4 of the bucket of chain 16 i + l / 4; the quad folds its four parts (DPP xor), the owner reads it back.
__global__ void k_coop4(const uint4* __restrict__ t, uint32_t nb, uint32_t iters, unsigned* out) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t s = mix(blockIdx.x * blockDim.x + threadIdx.x + 1u);
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t b = (uint32_t)(((uint64_t)s * nb) >> 32);  // this lane's own chain's bucket
        uint32_t v[4];
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
            const uint32_t c = 16u * i + (lane >> 2);  // the chain served by this lane in instruction i
            const uint32_t bc = (uint32_t)__shfl((int)b, (int)c);
            const uint4 a = t[4ull * bc + (lane & 3u)];
            uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
            x ^= (uint32_t)__shfl_xor((int)x, 1);
            x ^= (uint32_t)__shfl_xor((int)x, 2);
            v[i] = x;
        }
        // the owner lane o = 16 i + q reads the fold of quad q of instruction i
        const uint32_t q = lane & 15u, i0 = lane >> 4;
        uint32_t y = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
            const uint32_t yi = (uint32_t)__shfl((int)v[i], (int)(4u * q));
            y = i == i0 ? yi : y;
        }
        s = mix(s ^ y);
    }
    if (s == 0x12345678u) out[0] = s;
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 16;
    const uint32_t iters = argc > 2 ? (uint32_t)std::strtoul(argv[2], nullptr, 10) : 200;
    const size_t bytes = mib << 20;
    const uint32_t nb = (uint32_t)(bytes / 64);
    uint4* t = nullptr;
    unsigned* out = nullptr;
    CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(t, 0x5A, bytes));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const uint32_t grid = 5u * (uint32_t)p.multiProcessorCount;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double lookups = (double)grid * 256.0 * iters;
    for (int pat = 0; pat < 2; ++pat) {
        float best = 1e30f;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(e0));
            if (pat == 0) hipLaunchKernelGGL(k_lane64, dim3(grid), dim3(256), 0, 0, t, nb, iters, out);
            else hipLaunchKernelGGL(k_coop4, dim3(grid), dim3(256), 0, 0, t, nb, iters, out);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0 && ms < best) best = ms;
        }
        std::printf("{\"pattern\": \"%s\", \"table_mib\": %zu, \"iters\": %u, \"ms\": %.4f, \"G_lookups_s\": %.2f}\n",
                    pat == 0 ? "lane64" : "coop4", mib, iters, best, lookups / best / 1e6);
    }
    return 0;
}
