// Device-side building blocks shared by the scan translation units (scan_kernels.hip, ax_scan.hip): the index
// view, the LF-step search and classification helpers, and the host-side HIP helpers. DESIGN.md §3-§4.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "speq_errors.hpp"

namespace speq_dev {


constexpr uint32_t WAVES_PER_BLOCK = 4;
constexpr uint32_t BLOCK_THREADS = 64 * WAVES_PER_BLOCK;
constexpr uint32_t MAX_K = 4096;
constexpr uint32_t LDS_HIST_MAX_G = 2048;
constexpr uint32_t QLUT_LEN = 42;  // phred42 ranks 0..41
// local mode, per block in LDS: {1 - 10^(-q/10), its reciprocal} for q = 0..41, then (k_scan_kt) the weight of a window
// of k bases that all have quality q
constexpr uint32_t QTAB_BYTES = QLUT_LEN * 24u;

// a / b correctly rounded (IEEE division) from y = RN(1 / b) by two FMA corrections: q0 = a y is within 2 ulp, the
// first correction makes it faithful, and from a faithful quotient the second gives the correctly rounded one
// (Markstein). Bit-identical to `a / b` for the finite, normal operands of the Phred weights (b in [0.2, 1)).
__device__ __forceinline__ double div_rn(double a, double b, double y) {
    double q = a * y;
    double r = __fma_rn(-q, b, a);
    q = __fma_rn(r, y, q);
    r = __fma_rn(-q, b, a);
    return __fma_rn(r, y, q);
}

enum { KM_GLOBAL = 0, KM_LOCAL = 1, KM_REF = 2 };

struct DevView {
    const uint4* occ;        // 5 planes x n_blocks entries {C[s] + count, bits[3]}: A, C, G, T, N (plane-major)
    const uint4* occ2;       // 16 two-symbol planes x n_blocks (plane 4a+b), or null
    const uint4* occ3;       // 64 three-symbol planes x n_blocks (plane 16a+4b+c), or null (requires occ2)
    const uint4* runs;       // n_blocks entries over the label-change bitvector
    const uint16_t* run_label;
    const uint32_t* lab;     // per SA position {group | min(run_end - i, 65535) << 16}, or null
    const uint2* prefix;     // 4^q intervals (or null)
    const uint4* pfx_rank;   // sparse form of `prefix` (or null): {count, 96-bit presence} per 96 codes ...
    const uint2* pfx_iv;     // ... and the intervals of the present codes only, in code order
    const uint4* ktab;       // k-mer interval table for k == kt_k (or null): 64-B buckets of 4 slots, see KmerTable
    uint64_t kt_bmask;       // buckets - 1 (a power of two minus one); compact tables: the bucket count
    const uint2* kt_multi;   // compact tables: {lo, hi} of each multi-group k-mer
    uint32_t n, q, G, nb;
    uint32_t kt_k;
    uint32_t kt_compact;     // 1: ktab holds the compact 8-B-slot form (k <= KT8_MAX_K)
};

struct UnitSrc {
    const uint8_t* seq;       // reads: ASCII bases; ref: SA-alphabet text codes
    const uint8_t* qual;      // reads: Phred+33; ref: null
    const uint64_t* off;      // unit u spans [off[u], off[u+1] - end_adj)
    const uint64_t* cum_win;  // ref only: prefix sums of windows per text
    const int32_t* unit_group;  // ref only: group of each text
    const double* qlut;       // local only: {1 - 10^(-q/10), 1 / that} for q = 0..41
    uint32_t* em_mult;        // optional: per SA position, # passing multi-group windows whose interval starts there
    uint32_t* em_hi;          // optional: the end of that interval
    uint64_t n_units;         // reads (not pairs) or texts
    uint64_t total_windows;   // ref only: windows of this launch (a shard of the flattened reference windows)
    uint64_t win_base;        // ref only: first flattened window of the shard
    uint32_t end_adj;
    uint32_t k;
    uint32_t cutoff;
    uint32_t buf_bytes;       // per-wave staging buffer (bases)
    unsigned long long* ax_stats;  // diagnostic (speq_scan_reads_device_stats): k_scan_ax's work counters, else null
};

// Per-wave LDS: bases [buf_bytes] | qualities [buf_bytes] (local mode) | bad-mask words | N-mask words |
// base bit-plane words (bit 0 of every base's 2-bit code, then bit 1; k-mer table scans).
__host__ __device__ inline uint32_t staging_bytes(uint32_t k, uint32_t nwin) {
    return ((2u * (64u * nwin + k)) + 63u) & ~63u;
}
__host__ __device__ inline uint32_t mask_words(uint32_t buf) { return buf / 64u + 1u; }
__host__ __device__ inline uint32_t wave_lds_bytes(uint32_t buf, bool local) {
    return buf * (local ? 2u : 1u) + 32u * mask_words(buf);
}

__device__ __forceinline__ void wave_sync() {
    // Lanes of one wave exchange data through their wave-private LDS region: order the LDS writes before
    // the reads of other lanes (workgroup-scope fences emit the lgkmcnt wait).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rank_entry(u32x4 v, uint32_t r) {  // v.x + #bits set among the first r (0..96)
    const uint64_t a = (uint64_t)v[1] | ((uint64_t)v[2] << 32);
    const uint64_t ma = (r >= 64u) ? ~0ull : ((1ull << r) - 1ull);
    const uint32_t mb = (r <= 64u) ? 0u : ((r >= 96u) ? ~0u : ((1u << (r - 64u)) - 1u));
    return v[0] + (uint32_t)__popcll(a & ma) + (uint32_t)__popc(v[3] & mb);
}

// Buffer descriptors of the occ planes and of the run bitvector. A lane that does not need its second load of
// a step gets an out-of-range offset: the buffer range check drops that load (no memory request, returns 0), so
// both loads issue back to back with no branch and no wait on the first (a conditional plain load made hipcc
// wait for the first load before issuing the second).
struct Rsrc {
    __amdgpu_buffer_rsrc_t occ, occ2, occ3, runs;
};
constexpr uint32_t OOB = 0xFFFFFFF0u;
#ifndef SPEQ_HI_BRANCH
#define SPEQ_HI_BRANCH 0
#endif

__device__ __forceinline__ Rsrc make_rsrc(const DevView& I) {
    Rsrc R;
    R.occ = __builtin_amdgcn_make_buffer_rsrc((void*)I.occ, (short)0, (int)(5u * I.nb * 16u), 0x00020000);
    R.runs = __builtin_amdgcn_make_buffer_rsrc((void*)I.runs, (short)0, (int)(I.nb * 16u), 0x00020000);
    R.occ2 = __builtin_amdgcn_make_buffer_rsrc((void*)I.occ2, (short)0, I.occ2 ? (int)(16u * I.nb * 16u) : 0,
                                               0x00020000);
    R.occ3 = __builtin_amdgcn_make_buffer_rsrc((void*)I.occ3, (short)0, I.occ3 ? (int)(64u * I.nb * 16u) : 0,
                                               0x00020000);
    return R;
}

// Cache policy A/B knobs: read bytes are streamed once per launch, so loading them non-temporally keeps them from
// evicting index lines in L2; the q-mer table is one random 8-B load per window.
#ifndef SPEQ_NT_READS
#define SPEQ_NT_READS 0
#endif
#ifndef SPEQ_NT_PREFIX
#define SPEQ_NT_PREFIX 0
#endif
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
#if SPEQ_NT_READS
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
// q-mer interval of `code`: dense table, or (when 4^q is much larger than the number of distinct q-mers) a presence
// bitvector with ranks, L2-resident, plus the intervals of the present q-mers only. Absent q-mer: empty interval.
__device__ __forceinline__ uint2 ld_prefix(const uint2* p);
__device__ __forceinline__ uint2 prefix_lookup(const DevView& I, uint32_t code) {
    if (I.pfx_rank != nullptr) {
        const uint32_t b = code / 96u, r = code - b * 96u;
        const uint4 e = I.pfx_rank[b];
        const uint32_t word = r < 32u ? e.y : (r < 64u ? e.z : e.w);
        if (!((word >> (r & 31u)) & 1u)) return make_uint2(0u, 0u);
        const uint32_t bits[3] = {e.y, e.z, e.w};
        uint32_t c = e.x;
#pragma unroll
        for (uint32_t w = 0; w < 3; ++w) {
            const uint32_t lo = w * 32u;
            if (r >= lo + 32u) c += __popc(bits[w]);
            else if (r > lo) c += __popc(bits[w] & ((1u << (r - lo)) - 1u));
        }
        return I.pfx_iv[c];
    }
    return ld_prefix(I.prefix + code);
}
__device__ __forceinline__ uint2 ld_prefix(const uint2* p) {
#if SPEQ_NT_PREFIX
    const uint64_t v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p));
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
#else
    return *p;
#endif
}

// One backward-search step for both ends of [lo, hi): the two ranks share one 16-B load when they fall in the
// same 96-position block (narrow intervals, i.e. almost every step after the q-mer table). `rs` selects the
// one-symbol planes (plane = symbol) or the two-symbol planes (plane = 4a + b: extends by two bases).
__device__ __forceinline__ void lf_step(const DevView& I, __amdgpu_buffer_rsrc_t rs, uint32_t plane_id, uint32_t& lo,
                                        uint32_t& hi) {
    const uint32_t plane = plane_id * I.nb * 16u;
    const uint32_t bl = lo / 96u, bh = hi / 96u;
    const bool two = bh != bl;
#if SPEQ_HI_BRANCH  // A/B variant: exec-masked second load instead of the out-of-range offset
    u32x4 vx = {0u, 0u, 0u, 0u};
    if (two) vx = __builtin_amdgcn_raw_buffer_load_b128(rs, plane + bh * 16u, 0, 0);
    const u32x4 vl = __builtin_amdgcn_raw_buffer_load_b128(rs, plane + bl * 16u, 0, 0);
#else
    const u32x4 vl = __builtin_amdgcn_raw_buffer_load_b128(rs, plane + bl * 16u, 0, 0);
    const u32x4 vx = __builtin_amdgcn_raw_buffer_load_b128(rs, two ? plane + bh * 16u : OOB, 0, 0);
#endif
    const u32x4 vh = two ? vx : vl;
    lo = rank_entry(vl, lo - bl * 96u);  // entry counts include C[c]
    hi = rank_entry(vh, hi - bh * 96u);
}

// lf_step for a window that may be finished (lo >= hi): such a window issues no load and keeps its interval.
__device__ __forceinline__ void lf_step_pred(const DevView& I, __amdgpu_buffer_rsrc_t rs, uint32_t plane_id,
                                             uint32_t& lo, uint32_t& hi) {
    const bool act = lo < hi;
    const uint32_t plane = plane_id * I.nb * 16u;
    const uint32_t bl = lo / 96u, bh = hi / 96u;
    const bool two = bh != bl;
    const u32x4 vl = __builtin_amdgcn_raw_buffer_load_b128(rs, act ? plane + bl * 16u : OOB, 0, 0);
    const u32x4 vx = __builtin_amdgcn_raw_buffer_load_b128(rs, (act && two) ? plane + bh * 16u : OOB, 0, 0);
    const u32x4 vh = two ? vx : vl;
    const uint32_t nlo = rank_entry(vl, lo - bl * 96u), nhi = rank_entry(vh, hi - bh * 96u);
    lo = act ? nlo : lo;
    hi = act ? nhi : hi;
}

// Classifies a non-empty SA interval: run(i) = #label boundaries in [1, i]; one group <=> run(lo) == run(hi-1).
__device__ __forceinline__ int classify_runs(const DevView& I, const Rsrc& R, uint32_t lo, uint32_t hi) {
    const uint32_t last = hi - 1u;
    const uint32_t bl = lo / 96u, bh = last / 96u;
    const bool two = bh != bl;
    const u32x4 vl = __builtin_amdgcn_raw_buffer_load_b128(R.runs, bl * 16u, 0, 0);
    const u32x4 vx = __builtin_amdgcn_raw_buffer_load_b128(R.runs, two ? bh * 16u : OOB, 0, 0);
    const u32x4 vh = two ? vx : vl;
    const uint32_t rl = rank_entry(vl, lo - bl * 96u + 1u);
    const uint32_t rh = rank_entry(vh, last - bh * 96u + 1u);
    if (rl != rh) return -2;
    return (int)I.run_label[rl];
}

// One 4-B load when the label table is present: the run holding lo reaches hi-1 iff hi - lo <= its distance.
__device__ __forceinline__ int classify(const DevView& I, const Rsrc& R, uint32_t lo, uint32_t hi) {
    if (I.lab == nullptr) return classify_runs(I, R, lo, hi);
    const uint32_t x = I.lab[lo];
    const uint32_t dist = x >> 16, width = hi - lo;
    if (width <= dist) return (int)(x & 0xFFFFu);
    if (dist < 0xFFFFu) return -2;
    return classify_runs(I, R, lo, hi);  // saturated distance and a wider interval: exact rank path
}

// Exact backward search of the k symbols at w[0..k) (0..3 = ACGT, 4 = N) read from LDS (k > 32, or N in a
// reference window). Returns -1 (no occurrence), -2 (occurrences in >= 2 groups) or the single group id: the
// outcome of the first-hit rule at fm_scanner.cpp:165-177 when every record is assigned.
// The packed register form for k <= 32 is search_packed_n below.
__device__ __forceinline__ int search_lds(const DevView& I, const Rsrc& R, const unsigned char* w, uint32_t k,
                                          bool no_n, uint32_t& lo_out, uint32_t& hi_out) {
    uint32_t lo = 0, hi = I.n;
    int32_t s = (int32_t)k;
    if (I.q != 0u && k >= I.q) {
        uint32_t code = 0, bad = 0;
        for (uint32_t i = k - I.q; i < k; ++i) {
            const uint32_t c = w[i];
            bad |= c >> 2;
            code = (code << 2) | (c & 3u);
        }
        if (!bad) {
            const uint2 e = prefix_lookup(I, code);
            lo = e.x;
            hi = e.y;
            s -= (int32_t)I.q;
        }
    }
    if (I.occ3 != nullptr && no_n) {
        // s mod 3 leftover first (one single or one pair step), then three bases per step
        const int32_t rem = s % 3;
        if (rem == 1 && lo < hi) {
            lf_step(I, R.occ, w[s - 1], lo, hi);
            --s;
        } else if (rem == 2 && lo < hi) {
            lf_step(I, R.occ2, (uint32_t)w[s - 2] * 4u + w[s - 1], lo, hi);
            s -= 2;
        }
        while (s > 0 && lo < hi) {
            lf_step(I, R.occ3, (uint32_t)w[s - 3] * 16u + (uint32_t)w[s - 2] * 4u + w[s - 1], lo, hi);
            s -= 3;
        }
    } else if (I.occ2 != nullptr && no_n) {
        if ((s & 1) && lo < hi) {
            lf_step(I, R.occ, w[s - 1], lo, hi);
            --s;
        }
        while (s > 0 && lo < hi) {
            lf_step(I, R.occ2, (uint32_t)w[s - 2] * 4u + w[s - 1], lo, hi);
            s -= 2;
        }
    } else {
        uint32_t c = s > 0 ? w[s - 1] : 0u;
        while (s > 0 && lo < hi) {
            const uint32_t cn = s > 1 ? w[s - 2] : 0u;  // next symbol, read under this step's gathers
            lf_step(I, R.occ, c, lo, hi);
            c = cn;
            --s;
        }
    }
    lo_out = lo;
    hi_out = hi;
    return lo < hi ? classify(I, R, lo, hi) : -1;
}

__device__ __forceinline__ uint32_t ascii_sym(uint32_t ch) {  // dna5: A C G T/U -> 0..3, else N (4)
    // branch-free: ((x >> 1) ^ (x >> 2)) & 3 is 0 1 2 3 3 for a c g t u, and bits 0 2 6 19 20 of 0x180045 mark those
    // five letters at x - 'a' (any case; x = ch | 0x20)
    const uint32_t x = ch | 0x20u, d = x - 0x61u;
    const bool ok = d < 32u && ((0x180045u >> (d & 31u)) & 1u) != 0u;
    return ok ? (((x >> 1) ^ (x >> 2)) & 3u) : 4u;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// Backward search of NW windows per lane, interleaved so each lane keeps NW independent gather chains in flight
// (the kernel is bound by gather latency, not by L2 or fabric bandwidth: profiles/r01). Packed form only (k <= 32,
// no N). A window with an empty interval issues no further loads (out-of-range offsets).
template <int NW>
__device__ __forceinline__ void search_packed_n(const DevView& I, const Rsrc& R, const uint64_t (&P0)[NW],
                                                const bool (&act)[NW], uint32_t k, int (&out)[NW],
                                                uint32_t (&lo_out)[NW], uint32_t (&hi_out)[NW]) {
    uint64_t P[NW];
    uint32_t lo[NW], hi[NW];
    int32_t s = (int32_t)k;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        P[w] = P0[w];
        lo[w] = 0;
        hi[w] = act[w] ? I.n : 0u;
    }
    if (I.q != 0u && k >= I.q) {
        const uint64_t qmask = (1ull << (2u * I.q)) - 1ull;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            if (act[w]) {
                const uint2 e = prefix_lookup(I, (uint32_t)(P[w] & qmask));
                lo[w] = e.x;
                hi[w] = e.y;
            }
            P[w] >>= 2u * I.q;
        }
        s -= (int32_t)I.q;
    }
    if (I.occ3 != nullptr) {
        const int32_t rem = s % 3;  // leftover first: one single or one pair step
        if (rem == 1) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                lf_step_pred(I, R.occ, (uint32_t)(P[w] & 3u), lo[w], hi[w]);
                P[w] >>= 2;
            }
            --s;
        } else if (rem == 2) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                lf_step_pred(I, R.occ2, (uint32_t)(((P[w] >> 2) & 3u) * 4u + (P[w] & 3u)), lo[w], hi[w]);
                P[w] >>= 4;
            }
            s -= 2;
        }
        for (; s > 0; s -= 3) {
            bool any = false;
#pragma unroll
            for (int w = 0; w < NW; ++w) any |= lo[w] < hi[w];
            if (!any) break;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                // pattern becomes "a b c P": c = next symbol left of P (low bits), then b, then a
                const uint32_t plane = (uint32_t)(((P[w] >> 4) & 3u) * 16u + ((P[w] >> 2) & 3u) * 4u + (P[w] & 3u));
                lf_step_pred(I, R.occ3, plane, lo[w], hi[w]);
                P[w] >>= 6;
            }
        }
    } else if (I.occ2 != nullptr) {
        if (s & 1) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                lf_step_pred(I, R.occ, (uint32_t)(P[w] & 3u), lo[w], hi[w]);
                P[w] >>= 2;
            }
            --s;
        }
        for (; s > 0; s -= 2) {
            bool any = false;
#pragma unroll
            for (int w = 0; w < NW; ++w) any |= lo[w] < hi[w];
            if (!any) break;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                lf_step_pred(I, R.occ2, (uint32_t)(((P[w] >> 2) & 3u) * 4u + (P[w] & 3u)), lo[w], hi[w]);
                P[w] >>= 4;
            }
        }
    } else {
        for (; s > 0; --s) {
            bool any = false;
#pragma unroll
            for (int w = 0; w < NW; ++w) any |= lo[w] < hi[w];
            if (!any) break;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                lf_step_pred(I, R.occ, (uint32_t)(P[w] & 3u), lo[w], hi[w]);
                P[w] >>= 2;
            }
        }
    }
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        out[w] = (act[w] && lo[w] < hi[w]) ? classify(I, R, lo[w], hi[w]) : -1;
        lo_out[w] = lo[w];
        hi_out[w] = hi[w];
    }
}

#define HIP_OK(expr)                                                                                         \
    do {                                                                                                     \
        hipError_t _e = (expr);                                                                              \
        if (_e != hipSuccess)                                                                                \
            throw speq::DeviceError(std::string(#expr) + ": " + hipGetErrorString(_e));                      \
    } while (0)

// Host -> device copy of a pageable array. Large arrays are page-locked for the copy (hipHostRegister, ~3 ms for a
// 377 MB index) and copied by DMA at the link rate: the runtime's staged pageable copy ran at 2-10 GB/s, 0.24 s of a
// `speq scan` start-up (tools/upload_probe.cpp, profiles/r06/cli/). One registration at a time in the process (two
// replicas uploading the same host arrays must not unregister under each other's copy).
inline void upload_bytes(void* dst, const void* src, size_t bytes) {
    static std::mutex mu;
    if (bytes >= (4u << 20)) {
        std::lock_guard<std::mutex> lk(mu);
        if (hipHostRegister(const_cast<void*>(src), bytes, hipHostRegisterDefault) == hipSuccess) {
            const hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
            (void)hipHostUnregister(const_cast<void*>(src));
            HIP_OK(e);
            return;
        }
        (void)hipGetLastError();  // (not registered: the staged copy below)
    }
    HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
}

template <typename T>
T* dev_upload(const std::vector<T>& v) {
    if (v.empty()) return nullptr;
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, v.size() * sizeof(T)));
    upload_bytes(p, v.data(), v.size() * sizeof(T));
    return static_cast<T*>(p);
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        HIP_OK(hipGetDevice(&prev));
        if (prev != dev) HIP_OK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace speq_dev
