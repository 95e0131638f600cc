// GPU index construction: suffix array by prefix doubling on radix sorts, then BWT planes,
// two-symbol planes, label runs and the label table, all in HBM. Replaces the single-threaded SA construction of
// the reference's seqan3::fm_index{texts} (/root/reference/src/fm_indexer.cpp:36; SDSL upstream) and our host
// SA-IS for large collections (cfg 5: n = 200 M). Produces arrays bit-identical to the host build (fm_index.cpp),
// which tests check (tests/test_gpu_build.py).
//
// Suffix sorting (Manber-Myers doubling with Larsson-Sadakane style filtering):
//   round 0: key = first 21 symbols packed 3 bits each (63 bits), radix sort (key, suffix);
//   every suffix gets rank = SA position of the first member of its group of equal keys;
//   round r: only suffixes in groups of size > 1 stay active; key = (rank[i], rank[i + h]) for the current sorted
//   prefix length h, radix sort of the active list, scatter back into the group's slots, new ranks; h doubles.
// The collection's terminator is unique and smallest, so a suffix whose first h symbols include it is a singleton
// and every active suffix has i + h < n.
#include <hip/hip_runtime.h>

#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses ::memset

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fm_index.hpp"
#include "speq_errors.hpp"

namespace speq {
namespace {

#define BHIP(expr)                                                                                           \
    do {                                                                                                     \
        hipError_t _e = (expr);                                                                              \
        if (_e != hipSuccess) throw DeviceError(std::string("gpu build: ") + #expr + ": " + hipGetErrorString(_e)); \
    } while (0)

constexpr uint32_t KEY_SYMS = 21;  // 3 bits each

__global__ void k_init_keys(const uint8_t* __restrict__ T, uint32_t n, uint64_t* __restrict__ keys,
                            uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = 0;
#pragma unroll
    for (uint32_t j = 0; j < KEY_SYMS; ++j) {
        const uint32_t c = i + j < n ? T[i + j] : 0u;
        k = (k << 3) | c;
    }
    keys[i] = k;
    vals[i] = i;
}

// key of active suffix k = (rank[s] << bits) | rank[s + h]
__global__ void k_pair_keys(const uint32_t* __restrict__ act_suf, uint32_t m, const uint32_t* __restrict__ rank,
                            uint32_t n, uint32_t h, uint32_t bits, uint64_t* __restrict__ keys,
                            uint32_t* __restrict__ vals) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint32_t s = act_suf[k];
    const uint32_t r2 = s + h < n ? rank[s + h] : 0u;
    keys[k] = ((uint64_t)rank[s] << bits) | r2;
    vals[k] = s;
}

// head value for the max-scan: k if a new group starts at k (k == 0 or key differs), else 0
__global__ void k_heads(const uint64_t* __restrict__ keys, uint32_t m, uint32_t* __restrict__ hv) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    hv[k] = (k == 0 || keys[k] != keys[k - 1]) ? k : 0u;
}

// Scatters the sorted active list into its SA slots, assigns new ranks (slot of the group head), and flags the
// suffixes that remain in groups of size > 1. pos == nullptr means the identity (round 0).
__global__ void k_assign(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ suf,
                         const uint32_t* __restrict__ head_k, const uint32_t* __restrict__ pos, uint32_t m,
                         uint32_t* __restrict__ sa, uint32_t* __restrict__ rank, uint32_t* __restrict__ keep) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint32_t p = pos ? pos[k] : k;
    const uint32_t s = suf[k];
    sa[p] = s;
    const uint32_t hk = head_k[k];
    rank[s] = pos ? pos[hk] : hk;
    const bool head = k == 0 || keys[k] != keys[k - 1];
    const bool next_head = k + 1 == m || keys[k + 1] != keys[k];
    keep[k] = (head && next_head) ? 0u : 1u;
}

__global__ void k_compact(const uint32_t* __restrict__ keep, const uint32_t* __restrict__ off,
                          const uint32_t* __restrict__ pos, const uint32_t* __restrict__ suf, uint32_t m,
                          uint32_t* __restrict__ npos, uint32_t* __restrict__ nsuf) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m || !keep[k]) return;
    const uint32_t o = off[k];
    npos[o] = pos ? pos[k] : k;
    nsuf[o] = suf[k];
}

// BWT symbol, the symbol before it (0xFF when absent) and the group label of every SA position.
__global__ void k_bwt(const uint8_t* __restrict__ T, const uint32_t* __restrict__ sa, uint32_t n,
                      const uint64_t* __restrict__ text_start, uint32_t n_texts, const int32_t* __restrict__ text_group,
                      uint8_t* __restrict__ bwt, uint8_t* __restrict__ bwt2, uint8_t* __restrict__ code3,
                      uint16_t* __restrict__ label) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = sa[i];
    bwt[i] = s == 0 ? (uint8_t)SYM_TERM : T[s - 1];
    bwt2[i] = s >= 2 ? T[s - 2] : (uint8_t)0xFF;
    if (code3) {  // 16a + 4b + c for the three symbols before the suffix, 0xFF unless all are in A..T
        uint8_t c = 0xFF;
        if (s >= 3) {
            const uint32_t x = T[s - 3], y = T[s - 2], z = T[s - 1];
            if (x - SYM_A < 4u && y - SYM_A < 4u && z - SYM_A < 4u)
                c = (uint8_t)((x - SYM_A) * 16u + (y - SYM_A) * 4u + (z - SYM_A));
        }
        code3[i] = c;
    }
    // largest t with text_start[t] <= s, clamped to the last text (the terminator)
    uint32_t lo = 0, hi = n_texts + 1;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (text_start[mid] <= s) lo = mid;
        else hi = mid;
    }
    if (lo >= n_texts) lo = n_texts - 1;
    label[i] = (uint16_t)text_group[lo];
}

enum PlaneKind { PK_OCC = 0, PK_OCC2 = 1, PK_RUNS = 2, PK_OCC3 = 3 };

// One thread per (plane, 96-position block): bitmap + popcount.
template <int KIND>
__global__ void k_planes(const uint8_t* __restrict__ bwt, const uint8_t* __restrict__ bwt2,
                         const uint16_t* __restrict__ label, uint32_t n, uint32_t nb, uint32_t n_planes,
                         OccEntry* __restrict__ planes, uint32_t* __restrict__ pops) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nb * n_planes) return;
    const uint32_t plane = (uint32_t)(t / nb), b = (uint32_t)(t % nb);
    uint32_t bits[3] = {0, 0, 0}, pop = 0;
    for (uint32_t r = 0; r < OCC_BLOCK; ++r) {
        const uint64_t i = (uint64_t)b * OCC_BLOCK + r;
        if (i >= n) break;
        bool on;
        if (KIND == PK_OCC) {
            on = bwt[i] == SYM_A + plane;
        } else if (KIND == PK_OCC2) {
            on = bwt2[i] == SYM_A + plane / 4 && bwt[i] == SYM_A + plane % 4;
        } else if (KIND == PK_OCC3) {
            on = bwt2[i] == plane;  // bwt2 carries code3 for this kind
        } else {
            on = i > 0 && label[i] != label[i - 1];
        }
        if (on) {
            bits[r >> 5] |= 1u << (r & 31);
            ++pop;
        }
    }
    OccEntry e;
    e.count = 0;
    e.bits[0] = bits[0];
    e.bits[1] = bits[1];
    e.bits[2] = bits[2];
    planes[t] = e;
    pops[t] = pop;
}

__global__ void k_fold_counts(OccEntry* __restrict__ planes, const uint32_t* __restrict__ excl, uint64_t total,
                              uint32_t nb, const uint32_t* __restrict__ base) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    planes[t].count = excl[t] + base[t / nb];
}

__global__ void k_run_flags(const uint16_t* __restrict__ label, uint32_t n, uint32_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flag[i] = (i > 0 && label[i] != label[i - 1]) ? 1u : 0u;
}

// run id of i = inclusive prefix of flags; starts[run] = i where a run begins
__global__ void k_run_starts(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ run_id, uint32_t n,
                             const uint16_t* __restrict__ label, uint32_t* __restrict__ starts,
                             uint16_t* __restrict__ run_label) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == 0 || flag[i]) {
        starts[run_id[i]] = i;
        run_label[run_id[i]] = label[i];
    }
}

__global__ void k_lab(const uint16_t* __restrict__ label, const uint32_t* __restrict__ run_id,
                      const uint32_t* __restrict__ starts, uint32_t n, uint32_t* __restrict__ lab) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t end = starts[run_id[i] + 1];
    const uint32_t rem = min(end - i, 0xFFFFu);
    lab[i] = (uint32_t)label[i] | (rem << 16);
}

inline uint32_t grid(uint64_t n, uint32_t bs = 256) { return (uint32_t)((n + bs - 1) / bs); }

template <typename T>
struct DevBuf {
    T* p = nullptr;
    explicit DevBuf(uint64_t count) { BHIP(hipMalloc(&p, std::max<uint64_t>(count, 1) * sizeof(T))); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

struct Temp {
    void* p = nullptr;
    size_t bytes = 0;
    void need(size_t b) {
        if (b <= bytes) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        BHIP(hipMalloc(&p, b));
        bytes = b;
    }
    ~Temp() {
        if (p) (void)hipFree(p);
    }
};

uint32_t bits_for(uint64_t v) {
    uint32_t b = 1;
    while ((uint64_t(1) << b) <= v) ++b;
    return b;
}

}  // namespace

// Suffix array of the device text d_text[0, n) (SA alphabet codes; a unique smallest terminator at n - 1) into d_sa, on
// stream st (synchronous: the rounds read the survivor count back). Temporary device memory: about 52 B per symbol.
// Used by the index build below and by the anchor-structure build (ax_scan.hip: median representatives).
void gpu_suffix_sort(const uint8_t* d_text, uint32_t n, uint32_t* d_sa, void* stream, bool timing) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    DevBuf<uint32_t> d_rank(n);
    Temp tmp;
    {
        DevBuf<uint64_t> k0(n), k1(n);
        DevBuf<uint32_t> v0(n), v1(n), head(n), keep(n), off(n), pos0(n), pos1(n), suf0(n);
        // round 0
        k_init_keys<<<grid(n), 256, 0, st>>>(d_text, n, k0.p, v0.p);
        BHIP(hipGetLastError());
        rocprim::double_buffer<uint64_t> kb(k0.p, k1.p);
        rocprim::double_buffer<uint32_t> vb(v0.p, v1.p);
        size_t need = 0;
        BHIP(rocprim::radix_sort_pairs(nullptr, need, kb, vb, n, 0, 3 * KEY_SYMS, st));
        tmp.need(need);
        BHIP(rocprim::radix_sort_pairs(tmp.p, need, kb, vb, n, 0, 3 * KEY_SYMS, st));
        uint32_t m = n;
        const uint32_t* cur_pos = nullptr;  // SA slots of the active list; nullptr = identity (round 0)
        uint32_t h = KEY_SYMS;
        const uint32_t rb = bits_for(n);
        uint32_t rounds = 0;
        for (;;) {
            ++rounds;
            // groups of equal keys in the sorted active list: head slot by max-scan, ranks, survivors
            k_heads<<<grid(m), 256, 0, st>>>(kb.current(), m, head.p);
            BHIP(hipGetLastError());
            BHIP(rocprim::inclusive_scan(nullptr, need, head.p, head.p, m, rocprim::maximum<uint32_t>(), st));
            tmp.need(need);
            BHIP(rocprim::inclusive_scan(tmp.p, need, head.p, head.p, m, rocprim::maximum<uint32_t>(), st));
            k_assign<<<grid(m), 256, 0, st>>>(kb.current(), vb.current(), head.p, cur_pos, m, d_sa, d_rank.p,
                                              keep.p);
            BHIP(hipGetLastError());
            BHIP(rocprim::exclusive_scan(nullptr, need, keep.p, off.p, 0u, m, rocprim::plus<uint32_t>(), st));
            tmp.need(need);
            BHIP(rocprim::exclusive_scan(tmp.p, need, keep.p, off.p, 0u, m, rocprim::plus<uint32_t>(), st));
            uint32_t last_off = 0, last_keep = 0;
            // on st: the caller's stream may be a non-blocking one (the replica's), which hipMemcpy does not wait for
            BHIP(hipMemcpyAsync(&last_off, off.p + (m - 1), 4, hipMemcpyDeviceToHost, st));
            BHIP(hipMemcpyAsync(&last_keep, keep.p + (m - 1), 4, hipMemcpyDeviceToHost, st));
            BHIP(hipStreamSynchronize(st));
            const uint32_t m2 = last_off + last_keep;
            if (m2 == 0) break;
            if (h >= n) throw std::runtime_error("gpu build: suffix sorting did not converge");
            // compact the survivors: slots alternate between two buffers (the current ones are being read)
            uint32_t* npos = cur_pos == pos0.p ? pos1.p : pos0.p;
            k_compact<<<grid(m), 256, 0, st>>>(keep.p, off.p, cur_pos, vb.current(), m, npos, suf0.p);
            BHIP(hipGetLastError());
            m = m2;
            cur_pos = npos;
            // next round: sort the survivors by (rank[s], rank[s + h]), i.e. by their first 2h symbols
            k_pair_keys<<<grid(m), 256, 0, st>>>(suf0.p, m, d_rank.p, n, h, rb, kb.current(), vb.current());
            BHIP(hipGetLastError());
            BHIP(rocprim::radix_sort_pairs(nullptr, need, kb, vb, m, 0, 2 * rb, st));
            tmp.need(need);
            BHIP(rocprim::radix_sort_pairs(tmp.p, need, kb, vb, m, 0, 2 * rb, st));
            h *= 2;
        }
        if (timing) std::fprintf(stderr, "fm_build[gpu]: %u doubling rounds\n", rounds);
    }
}

// Fills idx.sa, occ, occ2 (pair_steps), runs, run_label and lab (label_table) from idx.text, idx.C, text_start and
// text_group, on `device`. The caller has built the text and C and builds the prefix table afterwards.
void fm_build_arrays_gpu(FmIndex& idx, int device, bool pair_steps, bool triple_steps, bool label_table,
                         bool timing) {
    auto t_last = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!timing) return;
        BHIP(hipDeviceSynchronize());
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "fm_build[gpu]: %-10s %.3f s\n", what, std::chrono::duration<double>(t - t_last).count());
        t_last = t;
    };
    int prev = -1;
    BHIP(hipGetDevice(&prev));
    BHIP(hipSetDevice(device));
    struct Restore {
        int d;
        ~Restore() {
            if (d >= 0) (void)hipSetDevice(d);
        }
    } restore{prev};
    hipStream_t st = nullptr;  // null stream: every step is ordered

    const uint64_t n64 = idx.n;
    if (n64 >= (uint64_t(1) << 31)) throw std::invalid_argument("gpu build: collection exceeds 2^31 symbols");
    const uint32_t n = (uint32_t)n64;
    const uint32_t nb = (uint32_t)idx.n_blocks();

    DevBuf<uint8_t> d_text(n);
    BHIP(hipMemcpy(d_text.p, idx.text.data(), n, hipMemcpyHostToDevice));
    DevBuf<uint32_t> d_sa(n);
    gpu_suffix_sort(d_text.p, n, d_sa.p, st, timing);
    Temp tmp;  // rocPRIM scratch of the steps below
    phase("sa");

    idx.sa.resize(n);
    BHIP(hipMemcpy(idx.sa.data(), d_sa.p, (size_t)n * 4, hipMemcpyDeviceToHost));

    DevBuf<uint64_t> d_ts(idx.text_start.size());
    DevBuf<int32_t> d_tg(idx.text_group.size());
    BHIP(hipMemcpy(d_ts.p, idx.text_start.data(), idx.text_start.size() * 8, hipMemcpyHostToDevice));
    BHIP(hipMemcpy(d_tg.p, idx.text_group.data(), idx.text_group.size() * 4, hipMemcpyHostToDevice));
    DevBuf<uint8_t> d_bwt(n), d_bwt2(n), d_code3(triple_steps ? n : 1);
    DevBuf<uint16_t> d_label(n);
    k_bwt<<<grid(n), 256, 0, st>>>(d_text.p, d_sa.p, n, d_ts.p, idx.n_texts, d_tg.p, d_bwt.p, d_bwt2.p,
                                   triple_steps ? d_code3.p : nullptr, d_label.p);
    BHIP(hipGetLastError());

    // planes: bitmaps + popcounts, one exclusive scan per plane, counts = scan + base (C[s] / C2[ab] / 0)
    auto build_planes = [&](int kind, uint32_t n_planes, const std::vector<uint32_t>& base,
                            std::vector<OccEntry>& out) {
        const uint64_t total = (uint64_t)nb * n_planes;
        DevBuf<OccEntry> d_pl(total);
        DevBuf<uint32_t> d_pop(total), d_ex(total), d_base(n_planes);
        const uint32_t g = grid(total);
        if (kind == PK_OCC)
            k_planes<PK_OCC><<<g, 256, 0, st>>>(d_bwt.p, d_bwt2.p, d_label.p, n, nb, n_planes, d_pl.p, d_pop.p);
        else if (kind == PK_OCC2)
            k_planes<PK_OCC2><<<g, 256, 0, st>>>(d_bwt.p, d_bwt2.p, d_label.p, n, nb, n_planes, d_pl.p, d_pop.p);
        else if (kind == PK_OCC3)
            k_planes<PK_OCC3><<<g, 256, 0, st>>>(d_bwt.p, d_code3.p, d_label.p, n, nb, n_planes, d_pl.p, d_pop.p);
        else
            k_planes<PK_RUNS><<<g, 256, 0, st>>>(d_bwt.p, d_bwt2.p, d_label.p, n, nb, n_planes, d_pl.p, d_pop.p);
        BHIP(hipGetLastError());
        for (uint32_t pl = 0; pl < n_planes; ++pl) {
            size_t need = 0;
            BHIP(rocprim::exclusive_scan(nullptr, need, d_pop.p + (uint64_t)pl * nb, d_ex.p + (uint64_t)pl * nb, 0u,
                                         nb, rocprim::plus<uint32_t>(), st));
            tmp.need(need);
            BHIP(rocprim::exclusive_scan(tmp.p, need, d_pop.p + (uint64_t)pl * nb, d_ex.p + (uint64_t)pl * nb, 0u,
                                         nb, rocprim::plus<uint32_t>(), st));
        }
        BHIP(hipMemcpy(d_base.p, base.data(), n_planes * 4, hipMemcpyHostToDevice));
        k_fold_counts<<<g, 256, 0, st>>>(d_pl.p, d_ex.p, total, nb, d_base.p);
        BHIP(hipGetLastError());
        out.resize(total);
        BHIP(hipMemcpy(out.data(), d_pl.p, total * sizeof(OccEntry), hipMemcpyDeviceToHost));
    };
    {
        std::vector<uint32_t> base(5);
        for (uint32_t s = 0; s < 5; ++s) base[s] = idx.C[SYM_A + s];
        build_planes(PK_OCC, 5, base, idx.occ);
    }
    phase("occ");
    if (pair_steps) {
        // C2[ab] = C[a] + #positions p with T[p] == a and T[p+1] < b
        uint64_t pc[SYM_COUNT][SYM_COUNT] = {{0}};
        const uint8_t* T = idx.text.data();
        for (uint64_t p = 0; p + 1 < n64; ++p) pc[T[p]][T[p + 1]]++;
        std::vector<uint32_t> base(16);
        for (uint8_t a = SYM_A; a <= SYM_T; ++a)
            for (uint8_t b = SYM_A; b <= SYM_T; ++b) {
                uint64_t c2 = idx.C[a];
                for (uint8_t c = 0; c < b; ++c) c2 += pc[a][c];
                base[(a - SYM_A) * 4 + (b - SYM_A)] = (uint32_t)c2;
            }
        build_planes(PK_OCC2, 16, base, idx.occ2);
    } else {
        idx.occ2.clear();
    }
    phase("occ2");
    if (triple_steps) {
        std::vector<uint32_t> base(64);
        triple_bases(idx, base.data());
        build_planes(PK_OCC3, 64, base, idx.occ3);
    } else {
        idx.occ3.clear();
    }
    phase("occ3");
    build_planes(PK_RUNS, 1, std::vector<uint32_t>(1, 0u), idx.runs);
    {
        DevBuf<uint32_t> flag(n), run_id(n);
        k_run_flags<<<grid(n), 256, 0, st>>>(d_label.p, n, flag.p);
        BHIP(hipGetLastError());
        size_t need = 0;
        BHIP(rocprim::inclusive_scan(nullptr, need, flag.p, run_id.p, n, rocprim::plus<uint32_t>(), st));
        tmp.need(need);
        BHIP(rocprim::inclusive_scan(tmp.p, need, flag.p, run_id.p, n, rocprim::plus<uint32_t>(), st));
        uint32_t last = 0;
        BHIP(hipMemcpy(&last, run_id.p + (n - 1), 4, hipMemcpyDeviceToHost));
        const uint32_t n_runs = last + 1;
        DevBuf<uint32_t> starts(n_runs + 1);
        DevBuf<uint16_t> rl(n_runs);
        k_run_starts<<<grid(n), 256, 0, st>>>(flag.p, run_id.p, n, d_label.p, starts.p, rl.p);
        BHIP(hipGetLastError());
        BHIP(hipMemcpy(starts.p + n_runs, &n, 4, hipMemcpyHostToDevice));
        idx.run_label.resize(n_runs);
        BHIP(hipMemcpy(idx.run_label.data(), rl.p, (size_t)n_runs * 2, hipMemcpyDeviceToHost));
        if (label_table) {
            DevBuf<uint32_t> lab(n);
            k_lab<<<grid(n), 256, 0, st>>>(d_label.p, run_id.p, starts.p, n, lab.p);
            BHIP(hipGetLastError());
            idx.lab.resize(n);
            BHIP(hipMemcpy(idx.lab.data(), lab.p, (size_t)n * 4, hipMemcpyDeviceToHost));
        } else {
            idx.lab.clear();
        }
    }
    BHIP(hipDeviceSynchronize());
    phase("labels");
}

}  // namespace speq

namespace speq {
// Loads this translation unit's code object onto the current device (HIP loads a code object at the first use of
// one of its kernels: 30-55 ms for the scan kernels' on the first launch of a `speq scan` run; speq_device_warmup).
void warm_module_build_gpu() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_init_keys));
}
}  // namespace speq
