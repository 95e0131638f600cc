// HIP kernels of the SPeQ scan path for gfx950 (MI355X), plus the device half of the C ABI.
//
// One kernel template serves the three reference loops that call seqan3::search:
//   KM_GLOBAL : read scan, integer tallies        /root/reference/src/fm_scanner.cpp:145-216 (paired :662-732)
//   KM_LOCAL  : read scan, Phred-weighted tallies /root/reference/src/fm_scanner.cpp:418-491 (paired :911-998)
//   KM_REF    : reference-uniqueness (.dat) pass  /root/reference/src/fm_scanner.cpp:1499-1542
//
// Work decomposition: a wavefront owns a contiguous range of units (reads, mate pairs, or a
// slice of reference windows) and walks the FLATTENED stream of their k-mer windows 64 at a time, one
// window per lane, so the short tail of one read is packed with the head of the next (130 windows per
// 150-bp read at k=21 would waste a third of the lanes with one read per pass). Per pass:
//   1. cursor: every lane loads the window count of read (r + lane) — one coalesced load — and a wave
//      prefix sum assigns lanes to (read, offset);
//   2. staging: the bases of the pass are loaded once (coalesced bytes) into a wave-private LDS buffer as
//      3-bit symbols; a ballot per 64 bases builds the "bad" bitmask (Phred <= cutoff or N, fm_scanner.cpp:162),
//      so a window's filter is one or two masked 64-bit tests;
//   3. search: exact LF-mapping backward search, one 16-B occ entry per rank, with the lo and hi ranks of a
//      step sharing ONE load whenever both fall in the same 96-position block;
//   4. classify: the SA interval holds one group iff it holds no label-run boundary (two rank loads, again
//      shared when in one block, and one run-label load);
//   5. tally into an LDS histogram (flushed with one global atomic per group per workgroup); read ambiguity
//      (fm_scanner.cpp:183-190, :709-729) is a segmented min/max scan across the lanes of each unit.
#include <hip/hip_runtime.h>

#include <chrono>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "capi_internal.hpp"
#include "em.hpp"
#include "scan_internal.hpp"
#include "fm_index.hpp"

#include "scan_device.hpp"
#include "device_index.hpp"

namespace {

using namespace speq_dev;


// ---- k-mer interval table (the q-mer table taken to q = k; built per k by k_ktab_keys + k_ktab_fill) ----
// Open addressing over 64-B buckets of four 16-B slots {key lo, key hi, lo, info}: key = the k-mer's two bit planes
// (bit j of the low word = bit 0 of base j's 2-bit code, bit j of the high word = its bit 1; k <= 31, so bit 31 of
// both words is clear and the all-ones key marks an empty slot), lo = start of its SA interval, info = its
// classification: the group id, or 0x80000000 | (hi - lo) when the occurrences span >= 2 groups. Every distinct
// N-free k-mer of the reference texts is present; a k-mer that is absent from the table does not occur. Keys are
// placed by linear probing over buckets, slots in order, without deletions, so a lookup that meets an empty slot
// before its key has proven the key absent. A scan reads a window's key straight from the ballots of its bases.
constexpr uint32_t KT_MAX_K = 31;
constexpr unsigned long long KT_EMPTY = ~0ull;
#ifndef SPEQ_KT_BSLOTS  // slots per bucket (A/B knob): a lookup reads 16 * SPEQ_KT_BSLOTS bytes
#define SPEQ_KT_BSLOTS 4
#endif
constexpr uint32_t KT_BSLOTS = SPEQ_KT_BSLOTS;

__host__ __device__ __forceinline__ uint32_t kt_hash(uint64_t key) {  // two 31-bit planes -> 32-bit bucket hash
    uint32_t x = (uint32_t)key ^ ((uint32_t)(key >> 32) * 0x9E3779B1u);
    x ^= x >> 16;  // murmur3 fmix32
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

// Bits [off, off + k) of a wave's plane words (k <= 31): bit j = base off + j.
__device__ __forceinline__ uint64_t plane_bits(const unsigned long long* pl, uint32_t off, uint32_t k) {
    // branch-free (no divergent path): the second word is read only when the bits straddle it
    const uint32_t w0 = off >> 6, sh = off & 63u;
    const bool two = sh + k > 64u;
    const uint64_t lo = pl[w0], hi = pl[w0 + (two ? 1u : 0u)];
    const uint64_t v = (lo >> sh) | (two ? ((hi << 1) << (63u - sh)) : 0ull);
    return v & ((1ull << k) - 1ull);
}

// plane_bits for k_scan_kt's LDS words: both words are always read (one ds_read2_b64; the arrays hold >= 4 words and a
// pass never starts a window past word 2), then selected without a branch.
__device__ __forceinline__ uint64_t plane_bits2(const unsigned long long* pl, uint32_t off, uint32_t k) {
    const uint32_t w0 = off >> 6, sh = off & 63u;
    const uint64_t lo = pl[w0], hi = pl[w0 + 1u];
    const uint64_t v = (lo >> sh) | (sh + k > 64u ? ((hi << 1) << (63u - sh)) : 0ull);
    return v & ((1ull << k) - 1ull);
}

// The packed code (2 bits per base, last base lowest: the form search_packed_n takes) of a plane key.
__device__ __forceinline__ uint64_t kt_code(uint64_t key, uint32_t k) {
    uint64_t code = 0;
    for (uint32_t j = 0; j < k; ++j)
        code = (code << 2) | ((key >> j) & 1ull) | (((key >> (32u + j)) & 1ull) << 1);
    return code;
}

// ---- compact k-mer table (k <= KT8_MAX_K): 64-B buckets of eight 8-B slots ----
// slot = ck << (64 - 2k) | payload with ck = plane0 | plane1 << k (the window's two bit planes, k bits each); payload = the
// group id, or (1 << (pb - 1)) | m for a k-mer whose occurrences span >= 2 groups, m indexing kt_multi[] = {lo, hi}
// (read by EM scans only); pb = 64 - 2k >= 18 bits. All-ones = empty (no valid payload is all ones). Any bucket count
// nb (bucket = mulhi(hash, nb)), so the table is sized for an exact load factor (kt_load8, 35 % by default: 7.3 MB at
// cfg 2) against 16 MB for the 16-B-slot form, small enough to stay mostly in L2.
constexpr uint32_t KT8_MAX_K = 23;
__host__ __device__ __forceinline__ uint32_t kt8_bucket(uint64_t key64, uint32_t nb) {
    return (uint32_t)(((uint64_t)kt_hash(key64) * nb) >> 32);
}
__host__ __device__ __forceinline__ uint64_t kt8_ck(uint64_t key64, uint32_t k) {
    return (key64 & 0xFFFFFFFFull) | ((key64 >> 32) << k);
}

// Same outputs as search_packed_n (group / -2 / -1 and, for -2, the SA interval) from one bucket load per window:
// the four slots are four independent 16-B loads of one 64-B line, issued together. A window whose bucket holds
// neither its key nor an empty slot probes the next bucket (rare at load factor <= 1/2).
template <int NW>
__device__ __forceinline__ void search_ktab_n(const DevView& I, const uint64_t (&P)[NW], const bool (&act)[NW],
                                              int (&out)[NW], uint32_t (&lo_out)[NW], uint32_t (&hi_out)[NW]) {
    uint32_t b[NW];
    bool pend[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        out[w] = -1;
        lo_out[w] = hi_out[w] = 0;
        pend[w] = act[w];
        b[w] = kt_hash(P[w]) & (uint32_t)I.kt_bmask;
    }
    for (;;) {
        bool any = false;
#pragma unroll
        for (int w = 0; w < NW; ++w) any |= pend[w];
        if (!any) break;
        u32x4 sl[NW][KT_BSLOTS];
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if (pend[w]) {
                const u32x4* p = reinterpret_cast<const u32x4*>(I.ktab) + b[w] * KT_BSLOTS;
#pragma unroll
                for (int j = 0; j < (int)KT_BSLOTS; ++j) sl[w][j] = p[j];
            }
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if (pend[w]) {
                const uint32_t kl = (uint32_t)P[w], kh = (uint32_t)(P[w] >> 32);
                bool empty = false, found = false;
                uint32_t lo = 0, info = 0;
#pragma unroll
                for (int j = 0; j < (int)KT_BSLOTS; ++j) {
                    const bool hit = sl[w][j][0] == kl && sl[w][j][1] == kh;
                    lo = hit ? sl[w][j][2] : lo;
                    info = hit ? sl[w][j][3] : info;
                    found |= hit;
                    empty |= sl[w][j][0] == 0xFFFFFFFFu && sl[w][j][1] == 0xFFFFFFFFu;
                }
                if (found) {
                    const bool multi = (info >> 31) != 0u;
                    out[w] = multi ? -2 : (int)info;
                    lo_out[w] = lo;
                    hi_out[w] = multi ? lo + (info & 0x7FFFFFFFu) : lo + 1u;  // single group: only lo is kept
                }
                pend[w] = !(found || empty);
                b[w] = (b[w] + 1u) & (uint32_t)I.kt_bmask;
            }
    }
}

#ifndef SPEQ_MIN_WAVES  // A/B knob: minimum waves per SIMD the register allocator must allow
#define SPEQ_MIN_WAVES 1
#endif
#ifndef SPEQ_KT_MIN_WAVES  // the same for global-mode k-mer-table scans, one window per lane: 6 waves/SIMD (<= 80 VGPRs)
#define SPEQ_KT_MIN_WAVES 6  // keep more lookups in flight (cfg 2: +9 %, profiles/r01/ab_kt_occupancy.jsonl)
#endif

// EM: also record the SA interval of every passing multi-group window (EM histogram scans only).
// KT: windows of k <= 31 are resolved in the k-mer interval table (I.ktab, I.kt_k == k) instead of by LF steps; a
// separate instantiation, so the LF-step kernel keeps its own register allocation.
template <int MODE, bool PAIRED, bool LDS_HIST, int NWIN, bool EM, bool KT>
__global__ __launch_bounds__(BLOCK_THREADS, (KT && NWIN == 1 && MODE == KM_GLOBAL) ? SPEQ_KT_MIN_WAVES : SPEQ_MIN_WAVES) void k_scan(DevView I, UnitSrc src, unsigned long long* __restrict__ out_a,
                                                        unsigned long long* __restrict__ out_b,
                                                        double* __restrict__ out_w) {
    // out_a: reads -> counts[G+2] (T, ambiguous, U[g]); ref -> U_ref[G]
    // out_b: ref -> Tot_ref[G];  out_w: local -> W[G]
    // A pass covers 64 * NWIN consecutive windows of the wave's stream: slot j = lane + 64 * w.
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = threadIdx.x & 63u;
    // the wave index is uniform: in an SGPR, so the wave's unit range, cursor and carried unit stay scalar and the
    // branches on them are uniform (no exec-mask bookkeeping)
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = I.G, k = src.k;
    // (+ 2 words: the workgroup's T and ambiguous units, flushed with the histogram: ax_scan.hip §4i)
    const uint32_t hist_words = LDS_HIST ? ((MODE == KM_GLOBAL) ? G : 2u * G) + 2u : 0u;
    const uint32_t hist_bytes = (hist_words * 8u + 15u) & ~15u;
    unsigned long long* hA = reinterpret_cast<unsigned long long*>(smem);
    unsigned long long* hT = hA + (hist_words >= 2u ? hist_words - 2u : 0u);  // LDS_HIST: {T, ambiguous}
    unsigned long long* hB = hA + G;              // KM_REF: Tot_ref
    double* hW = reinterpret_cast<double*>(hA + G);  // KM_LOCAL: W
    const uint32_t buf = src.buf_bytes;
    double2* qtab = reinterpret_cast<double2*>(smem + hist_bytes);  // KM_LOCAL only
    const uint32_t qtab_bytes = MODE == KM_LOCAL ? QTAB_BYTES : 0u;
    unsigned char* sbuf = smem + hist_bytes + qtab_bytes + wid * wave_lds_bytes(buf, MODE == KM_LOCAL);
    unsigned char* qbuf = sbuf + buf;
    unsigned long long* mbuf =
        reinterpret_cast<unsigned long long*>(sbuf + buf * (MODE == KM_LOCAL ? 2u : 1u));
    unsigned long long* nbuf = mbuf + mask_words(buf);  // KM_REF: N positions (windows with N search via LDS)
    unsigned long long* pbuf = nbuf + mask_words(buf);  // KT: bit 0 planes, then (+ mask_words) bit 1 planes
    const Rsrc R = make_rsrc(I);

    if (MODE == KM_LOCAL)
        for (uint32_t i = threadIdx.x; i < QLUT_LEN; i += BLOCK_THREADS)
            qtab[i] = make_double2(src.qlut[2 * i], src.qlut[2 * i + 1]);
    if (LDS_HIST)
        for (uint32_t i = threadIdx.x; i < hist_words; i += BLOCK_THREADS) hA[i] = 0ull;
    if (LDS_HIST || MODE == KM_LOCAL) __syncthreads();
    unsigned long long* gU = (MODE == KM_REF) ? out_a : out_a + 2;

    const uint64_t NW = (uint64_t)gridDim.x * WAVES_PER_BLOCK;
    const uint64_t gw = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + wid;
    uint64_t r, r_end, o = 0, remaining;
    if (MODE == KM_REF) {
        const uint64_t F0 = src.win_base + src.total_windows * gw / NW;
        const uint64_t F1 = src.win_base + src.total_windows * (gw + 1) / NW;
        remaining = F1 - F0;
        uint64_t lo = 0, hi = src.n_units;  // largest t with cum_win[t] <= F0
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (src.cum_win[mid] <= F0) lo = mid; else hi = mid;
        }
        r = lo;
        o = F0 - src.cum_win[lo];
        r_end = src.n_units;
    } else {
        const uint64_t nu = PAIRED ? src.n_units / 2 : src.n_units;
        const uint64_t u0 = nu * gw / NW, u1 = nu * (gw + 1) / NW;
        r = PAIRED ? 2 * u0 : u0;
        r_end = PAIRED ? 2 * u1 : u1;
        remaining = ~0ull;
    }

    uint32_t t_cnt = 0;       // passing windows seen by this lane
    uint32_t amb = 0;         // ambiguous units finished by this wave (wave-uniform)
    int cmin = INT_MAX, cmax = -1;
    uint64_t cunit = ~0ull;   // unit whose windows continue past the previous (sub-)pass

    while (r < r_end && remaining > 0) {
        // ---- 1. cursor: lane i holds the windows of read r+i still to scan (read r starts at window o).
        // Window counts are clamped to 64*NWIN+1: only the first 64*NWIN windows of the pass matter, and the
        // clamp keeps the lane prefix sums in 32 bits.
        uint32_t wl = 0;
        uint64_t bl_ = 0;
        if (r + lane < r_end) {
            bl_ = ld_stream(src.off + r + lane);
            const uint64_t L = ld_stream(src.off + r + lane + 1) - src.end_adj - bl_;
            uint64_t W = L >= k ? L - k + 1 : 0;
            if (lane == 0) W = W > o ? W - o : 0;
            wl = (uint32_t)(W < 64u * NWIN + 1u ? W : 64u * NWIN + 1u);
        }
        uint32_t incl = wl;  // inclusive prefix sum across lanes
        for (uint32_t d = 1; d < 64u; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t total = __shfl(incl, 63);
        if (total == 0) {  // the next 64 reads hold no window
            r = (r + 64 < r_end) ? r + 64 : r_end;
            o = 0;
            continue;
        }
        // slot j belongs to read r + ri, ri = #{reads whose windows end at or before j} (binary search over lanes)
        uint32_t ri[NWIN], oo[NWIN], off[NWIN];
        bool has[NWIN];
        uint64_t s0 = 0;
#pragma unroll
        for (int w = 0; w < NWIN; ++w) {
            const uint32_t slot = lane + 64u * (uint32_t)w;
            uint32_t i_lo = 0;
            for (uint32_t step = 32; step >= 1; step >>= 1) {
                const uint32_t v = __shfl(incl, (int)(i_lo + step - 1u));
                if (v <= slot) i_lo += step;
            }
            ri[w] = i_lo > 63u ? 63u : i_lo;
            const uint32_t excl_i = __shfl(incl, (int)ri[w]) - __shfl(wl, (int)ri[w]);
            oo[w] = slot - excl_i;  // window offset in the read, relative to o for read r (ri == 0)
            const uint64_t pos = __shfl(bl_, (int)ri[w]) + oo[w] + (ri[w] == 0 ? o : 0);
            if (w == 0) s0 = __shfl(pos, 0);
            off[w] = (uint32_t)(pos - s0);  // < buf for every slot that is taken
            has[w] = slot < total && pos + k - s0 <= buf && (uint64_t)slot < remaining;
        }
        uint32_t n_taken = 0, off_last = 0, ri_last = 0, oo_last = 0;
#pragma unroll
        for (int w = 0; w < NWIN; ++w) {
            const uint32_t c = (uint32_t)__popcll(__ballot(has[w]));  // valid slots are a prefix in slot order
            if (c > 0) {
                off_last = __shfl(off[w], (int)(c - 1u));
                ri_last = __shfl(ri[w], (int)(c - 1u));
                oo_last = __shfl(oo[w], (int)(c - 1u));
            }
            n_taken += c;
        }
        const uint32_t span = off_last + k;

        // ---- 2. stage bases [s0, s0 + span) into LDS; ballot the "bad" mask 64 bases at a time
        for (uint32_t p0 = 0; p0 < span; p0 += 64u) {
            const uint32_t p = p0 + lane;
            uint32_t bad = 1, isn = 0, sym = 0;
            if (p < span) {
                const uint32_t ch = ld_stream(src.seq + s0 + p);
                if (MODE == KM_REF) {
                    sym = ch - 2u;            // SA alphabet A..N = 2..6
                    bad = ch < 2u ? 1u : 0u;  // separator / terminator
                    isn = sym == 4u ? 1u : 0u;
                } else {
                    sym = ascii_sym(ch);
                    int q = (int)ld_stream(src.qual + s0 + p) - 33;
                    q = q < 0 ? 0 : (q > 41 ? 41 : q);
                    bad = ((uint32_t)q <= src.cutoff || sym == 4u) ? 1u : 0u;
                    if (MODE == KM_LOCAL) qbuf[p] = (unsigned char)q;
                }
                sbuf[p] = (unsigned char)sym;
            }
            const uint64_t m = __ballot(bad != 0u);
            if (lane == 0) mbuf[p0 >> 6] = m;
            if (KT) {  // the k-mer table key of a window is its two base bit planes (see kt_key)
                const uint64_t b0 = __ballot((sym & 1u) != 0u), b1 = __ballot((sym & 2u) != 0u);
                if (lane == 0) {
                    pbuf[p0 >> 6] = b0;
                    pbuf[mask_words(buf) + (p0 >> 6)] = b1;
                }
            }
            if (MODE == KM_REF) {
                const uint64_t nm = __ballot(isn != 0u);
                if (lane == 0) nbuf[p0 >> 6] = nm;
            }
        }
        wave_sync();

        // ---- 3./4. filter, search, classify
        int which[NWIN];
        uint32_t ilo[NWIN], ihi[NWIN];  // final SA interval (EM histogram)
        bool valid[NWIN], packed[NWIN];
        uint64_t P[NWIN];
#pragma unroll
        for (int w = 0; w < NWIN; ++w) {
            which[w] = -1;
            ilo[w] = ihi[w] = 0;
            valid[w] = false;
            packed[w] = false;
            P[w] = 0;
            if (has[w]) {
                const uint32_t w0 = off[w] >> 6, w1 = (off[w] + k - 1u) >> 6;
                uint64_t badbits = 0, nbits = 0;
                for (uint32_t wi = w0; wi <= w1; ++wi) {
                    uint64_t sel = ~0ull;
                    if (wi == w0) sel &= ~0ull << (off[w] & 63u);
                    if (wi == w1) sel &= ~0ull >> (63u - ((off[w] + k - 1u) & 63u));
                    badbits |= mbuf[wi] & sel;
                    if (MODE == KM_REF) nbits |= nbuf[wi] & sel;
                }
                valid[w] = badbits == 0;
                packed[w] = valid[w] && k <= 32u && nbits == 0;
                if (KT && packed[w]) {
                    P[w] = plane_bits(pbuf, off[w], k) | (plane_bits(pbuf + mask_words(buf), off[w], k) << 32);
                } else if (packed[w]) {
                    const unsigned char* ws = sbuf + off[w];
                    uint64_t x = 0;
                    for (uint32_t i = 0; i < k; ++i) x = (x << 2) | (uint64_t)(ws[i] & 3u);
                    P[w] = x;
                } else if (valid[w] && !(KT && MODE != KM_REF)) {  // KT read scans: k <= 31, no N -> packed
                    which[w] = search_lds(I, R, sbuf + off[w], k, nbits == 0, ilo[w], ihi[w]);
                }
            }
        }
        {
            int wp[NWIN];
            uint32_t plo[NWIN], phi[NWIN];
            if (KT) search_ktab_n<NWIN>(I, P, packed, wp, plo, phi);
            else search_packed_n<NWIN>(I, R, P, packed, k, wp, plo, phi);
#pragma unroll
            for (int w = 0; w < NWIN; ++w)
                if (packed[w]) {
                    which[w] = wp[w];
                    ilo[w] = plo[w];
                    ihi[w] = phi[w];
                }
        }

        // ---- 5. tallies
#pragma unroll
        for (int w = 0; w < NWIN; ++w) {
            if (MODE == KM_REF) {
                if (has[w] && valid[w]) {
                    const int g = src.unit_group[r + ri[w]];
                    if (LDS_HIST) {
                        atomicAdd(&hB[g], 1ull);
                        if (which[w] == g) atomicAdd(&hA[g], 1ull);
                    } else {
                        atomicAdd(&out_b[g], 1ull);
                        if (which[w] == g) atomicAdd(&out_a[g], 1ull);
                    }
                }
            } else if (valid[w]) {
                ++t_cnt;
                if (EM && which[w] == -2) {
                    // EM histogram: distinct k-mers have disjoint SA intervals, so lo
                    // identifies the interval; hi is the same for every window that hits it.
                    atomicAdd(&src.em_mult[ilo[w]], 1u);
                    src.em_hi[ilo[w]] = ihi[w];
                }
                if (which[w] >= 0) {
                    double wgt = 0.0;
                    if (MODE == KM_LOCAL) {
                        // w = 1.0; for q in window: w = w / (1 - 1/10^(q/10))   (fm_scanner.cpp:454, left to right)
                        const unsigned char* qw = qbuf + off[w];
                        double x = 1.0;
                        for (uint32_t i = 0; i < k; ++i) {
                            const double2 t = qtab[qw[i]];
                            x = div_rn(x, t.x, t.y);  // == x / t.x
                        }
                        wgt = x;
                    }
                    if (LDS_HIST) {
                        atomicAdd(&hA[which[w]], 1ull);
                        if (MODE == KM_LOCAL) atomicAdd(&hW[which[w]], wgt);
                    } else {
                        atomicAdd(&gU[which[w]], 1ull);
                        if (MODE == KM_LOCAL) atomicAdd(&out_w[which[w]], wgt);
                    }
                }
            }
        }
        if (MODE == KM_REF) remaining -= n_taken;

        // ---- 6. ambiguity: a unit is ambiguous iff its counted windows name >= 2 groups (min != max).
        // Sub-pass w covers slots [64w, 64w + 64) in stream order; the last unit of a sub-pass is carried.
        if (MODE != KM_REF) {
#pragma unroll
            for (int w = 0; w < NWIN; ++w) {
                const uint64_t hm = __ballot(has[w]);
                if (hm == 0) continue;
                const uint32_t last = (uint32_t)__popcll(hm) - 1u;
                const uint64_t unit = PAIRED ? ((r + ri[w]) >> 1) : (r + ri[w]);
                int vmin = (valid[w] && which[w] >= 0) ? which[w] : INT_MAX;
                int vmax = (valid[w] && which[w] >= 0) ? which[w] : -1;
                const uint64_t unit0 = __shfl(unit, 0);
                if (cunit != ~0ull && unit0 != cunit) {  // the carried unit is complete
                    amb += (cmax >= 0 && cmin != cmax) ? 1u : 0u;
                    cunit = ~0ull;
                }
                if (lane == 0 && unit == cunit) {
                    vmin = min(vmin, cmin);
                    vmax = max(vmax, cmax);
                }
                const uint64_t uprev = __shfl_up(unit, 1);
                const bool head = has[w] && (lane == 0 || unit != uprev);
                const uint64_t heads = __ballot(head);
                const uint64_t below = heads & ((lane == 63u) ? ~0ull : ((2ull << lane) - 1ull));
                const uint32_t seg_start = 63u - (uint32_t)__clzll(below);
                for (uint32_t d = 1; d < 64u; d <<= 1) {
                    const int om = __shfl_up(vmin, d), oM = __shfl_up(vmax, d);
                    if (lane >= d && lane - d >= seg_start) {
                        vmin = min(vmin, om);
                        vmax = max(vmax, oM);
                    }
                }
                const bool tail = has[w] && (lane == last || ((heads >> (lane + 1u)) & 1ull));
                const bool amb_lane = tail && lane != last && vmax >= 0 && vmin != vmax;
                amb += (uint32_t)__popcll(__ballot(amb_lane));
                cmin = __shfl(vmin, (int)last);
                cmax = __shfl(vmax, (int)last);
                cunit = __shfl(unit, (int)last);
            }
        }
        wave_sync();
        // ---- advance the cursor past the last window taken
        o = (ri_last == 0 ? o : 0) + oo_last + 1;
        r = r + ri_last;
    }

    if (MODE != KM_REF) {
        if (cunit != ~0ull) amb += (cmax >= 0 && cmin != cmax) ? 1u : 0u;
        const unsigned long long tsum = wave_sum<unsigned long long>((unsigned long long)t_cnt);
        if (lane == 0) {
            unsigned long long* tgt = LDS_HIST ? hT : out_a;
            if (tsum) atomicAdd(&tgt[0], tsum);
            if (amb) atomicAdd(&tgt[1], (unsigned long long)amb);
        }
    }
    if (LDS_HIST) {
        __syncthreads();
        if (MODE != KM_REF && threadIdx.x < 2u) {
            const unsigned long long x = hT[threadIdx.x];
            if (x) atomicAdd(&out_a[threadIdx.x], x);
        }
        for (uint32_t g = threadIdx.x; g < G; g += BLOCK_THREADS) {
            const unsigned long long a = hA[g];
            if (a) atomicAdd(&gU[g], a);
            if (MODE == KM_REF) {
                const unsigned long long b = hB[g];
                if (b) atomicAdd(&out_b[g], b);
            }
            if (MODE == KM_LOCAL) {
                const double x = hW[g];
                if (x != 0.0) atomicAdd(&out_w[g], x);
            }
        }
    }
}

// ---- software-pipelined k-mer-table read scan ----
// k_scan runs each pass of windows as three dependent global round trips (read offsets -> bases -> table), so a
// wave spends most of a pass waiting. k_scan_kt overlaps them across passes: while the table lookups of pass i are
// in flight, the offsets of pass i + 2 and the bases of pass i + 1 are already loading. Same results as k_scan
// (KM_GLOBAL / KM_LOCAL reads, paired or not, EM or not); the pass logic is k_scan's, with NW windows per lane.

// Wave-uniform lane reads (v_readlane: the result lives in a scalar register, unlike __shfl's ds_bpermute).
__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
__device__ __forceinline__ int rli(int v, uint32_t l) { return __builtin_amdgcn_readlane(v, (int)l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
    return (uint64_t)rl32((uint32_t)v, l) | ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32);
}

template <int NW>
struct KtCursor {
    uint64_t r, o;             // first unit of the pass and the window offset in it
    uint64_t s0;               // first base of the pass
    uint32_t ri[NW], oo[NW], off[NW];  // slot lane + 64 w: read r + ri, window oo of it, first base s0 + off
    uint32_t has[NW];          // the slot holds a window (0/1)
    uint32_t span, ri_last, oo_last;
    uint32_t any;              // the pass holds a window (0/1; wave-uniform)
    uint64_t units;            // bit i: unit r + i has windows in the pass (wave-uniform)
};

// Offsets of reads r + lane and r + lane + 1 (issued here, consumed by kt_cursor). Every lane loads (indices are
// clamped to the valid range off[0 .. r_end]): unconditional loads let the compiler count them, so a later wait for
// these does not also wait for the table lookups issued after them.
__device__ __forceinline__ void kt_load_offsets(const UnitSrc& src, uint64_t r, uint64_t r_end, uint32_t lane,
                                                uint64_t& b, uint64_t& e) {
    const uint64_t i = r + lane < r_end ? r + lane : r_end;
    b = src.off[i];
    e = src.off[i + 1 <= r_end ? i + 1 : r_end];
}

// bases a pass of k_scan_kt stages: NW + 1 chunks of 64 (windows past it wait for the next pass)
template <int NW>
__host__ __device__ constexpr uint32_t kt_span() { return 64u * (NW + 1); }

// The slots of a pass: units r, r+1, ... (lane i holds the window count of unit r + i) are walked in a wave-uniform
// loop over the units that have windows in the pass (one or two for 150-bp reads), each assigning its window range
// to the slots it covers: no prefix sum or per-slot binary search (those cost ~15 ds_bpermute per pass in k_scan).
template <int NW>
__device__ __forceinline__ KtCursor<NW> kt_cursor(uint64_t r, uint64_t o, uint64_t r_end, uint64_t bl_,
                                                  uint64_t el_, uint32_t lane, uint32_t k) {
    KtCursor<NW> c;
    c.r = r;
    c.o = o;
    uint32_t wl = 0;
    if (r + lane < r_end) {
        const uint64_t L = el_ - bl_;
        uint64_t W = L >= k ? L - k + 1 : 0;
        if (lane == 0) W = W > o ? W - o : 0;
        wl = (uint32_t)(W < 64u * NW + 1u ? W : 64u * NW + 1u);
    }
    uint64_t pos[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        c.ri[w] = c.oo[w] = 0;
        pos[w] = 0;
    }
    uint64_t nz = __ballot(wl != 0u);  // units with windows
    uint32_t start = 0;
    c.units = 0;
    while (nz != 0 && start < 64u * NW) {
        const uint32_t i = (uint32_t)__builtin_ctzll(nz);
        nz &= nz - 1;
        const uint32_t wi = rl32(wl, i);
        const uint64_t base = rl64(bl_, i) + (i == 0 ? o : 0);
        c.units |= 1ull << i;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t slot = lane + 64u * (uint32_t)w;
            const bool in = slot >= start && slot - start < wi;
            c.ri[w] = in ? i : c.ri[w];
            c.oo[w] = in ? slot - start : c.oo[w];
            pos[w] = in ? base + (slot - start) : pos[w];
        }
        start += wi;
    }
    const uint32_t total = start;
    c.any = total > 0 ? 1u : 0u;
    const uint64_t s0 = rl64(pos[0], 0);
    c.s0 = s0;
    uint32_t n_all = 0, last_w = 0, last_lane = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t slot = lane + 64u * (uint32_t)w;
        c.off[w] = (uint32_t)(pos[w] - s0);
        // valid slots are a prefix in slot order; the first window (pos == s0) always fits: k <= 31 < kt_span
        c.has[w] = (slot < total && pos[w] + k - s0 <= kt_span<NW>()) ? 1u : 0u;
        const uint32_t n = (uint32_t)__popcll(__ballot(c.has[w] != 0u));
        if (n > 0) {
            last_w = (uint32_t)w;
            last_lane = n - 1u;
        }
        n_all += n;
    }
    uint32_t off_last = 0;
    c.ri_last = c.oo_last = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w)
        if (n_all > 0 && last_w == (uint32_t)w) {
            off_last = rl32(c.off[w], last_lane);
            c.ri_last = rl32(c.ri[w], last_lane);
            c.oo_last = rl32(c.oo[w], last_lane);
        }
    c.span = off_last + k;
    return c;
}

// Where the pass after `c` starts (k_scan's cursor advance); a pass without windows skips 64 units.
template <int NW>
__device__ __forceinline__ void kt_advance(const KtCursor<NW>& c, uint64_t r_end, uint64_t& r, uint64_t& o) {
    if (!c.any) {
        r = (c.r + 64 < r_end) ? c.r + 64 : r_end;
        o = 0;
    } else {
        o = (c.ri_last == 0 ? c.o : 0) + c.oo_last + 1;
        r = c.r + c.ri_last;
    }
}

// One 64-base chunk of a k_scan_kt pass into LDS: qualities (local mode), the bad mask and the two base bit planes.
// Local mode also: the quality-change mask (bit p: q[p] != q[p - 1]; `qprev` = the previous chunk's last quality,
// updated here), so a window whose qualities are all equal takes its weight from a per-block table.
template <int MODE>
__device__ __forceinline__ void kt_stage_chunk(const UnitSrc& src, uint32_t ch, uint32_t qv, uint32_t p,
                                               uint32_t span, unsigned char* qbuf, unsigned long long* mbuf,
                                               unsigned long long* p0buf, unsigned long long* p1buf,
                                               unsigned long long* dbuf, uint32_t& qprev, uint32_t j) {
    // branch-free (the loads were clamped into the pass, so ch and qv are defined for every lane)
    const bool in = p < span;
    const uint32_t s5 = ascii_sym(ch);
    int q = (int)qv - 33;
    q = q < 0 ? 0 : (q > 41 ? 41 : q);
    const uint32_t sym = in ? s5 : 0u;
    const uint32_t bad = (!in || (uint32_t)q <= src.cutoff || s5 == 4u) ? 1u : 0u;
    if (!in) q = 0;
    if (MODE == KM_LOCAL && in) qbuf[p] = (unsigned char)q;
    const uint64_t m = __ballot(bad != 0u);
    const uint64_t b0 = __ballot((sym & 1u) != 0u), b1 = __ballot((sym & 2u) != 0u);
    uint64_t dm = 0;
    if (MODE == KM_LOCAL) {
        const uint32_t lane = p & 63u;
        int qp = __shfl_up(q, 1);
        if (lane == 0) qp = (int)qprev;
        dm = __ballot(q != qp);
        qprev = (uint32_t)__builtin_amdgcn_readlane(q, 63);
    }
    if ((p & 63u) == 0u) {
        mbuf[j] = m;
        p0buf[j] = b0;
        p1buf[j] = b1;
        if (MODE == KM_LOCAL) dbuf[j] = dm;
    }
}

// Staging registers of one pass: NW + 1 chunks of 64 bases; every lane loads (addresses clamped into the pass, or
// to `fallback`, a base of the current pass, when the pass is empty).
template <int NW>
struct KtStage {
    uint32_t c[NW + 1], q[NW + 1];
};
template <int NW>
__device__ __forceinline__ void kt_stage_load(const UnitSrc& src, const KtCursor<NW>& cu, uint64_t fallback,
                                              uint32_t lane, KtStage<NW>& st) {
    const uint64_t b = cu.any ? cu.s0 : fallback;
    const uint32_t l = cu.any ? cu.span - 1u : 0u;
#pragma unroll
    for (int j = 0; j <= NW; ++j) {
        const uint32_t p = min(64u * (uint32_t)j + lane, l);
        st.c[j] = ld_stream(src.seq + b + p);
        st.q[j] = ld_stream(src.qual + b + p);
    }
}

#ifndef SPEQ_KTP_MIN_WAVES
#define SPEQ_KTP_MIN_WAVES 1
#endif
#ifndef SPEQ_PROBE_NOLOOKUP
#define SPEQ_PROBE_NOLOOKUP 0
#endif
template <int MODE, bool PAIRED, bool LDS_HIST, bool EM, int NW, bool CK>
__global__ __launch_bounds__(BLOCK_THREADS, SPEQ_KTP_MIN_WAVES)
void k_scan_kt(DevView I, UnitSrc src, unsigned long long* __restrict__ out_a, double* __restrict__ out_w) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = threadIdx.x & 63u;
    // the wave index is uniform: in an SGPR, so the wave's unit range, cursor and carried unit stay scalar and the
    // branches on them are uniform (no exec-mask bookkeeping)
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = I.G, k = src.k;
    // (+ 2 words: the workgroup's T and ambiguous units, flushed with the histogram: ax_scan.hip §4i)
    const uint32_t hist_words = LDS_HIST ? ((MODE == KM_GLOBAL) ? G : 2u * G) + 2u : 0u;
    const uint32_t hist_bytes = (hist_words * 8u + 15u) & ~15u;
    unsigned long long* hA = reinterpret_cast<unsigned long long*>(smem);
    unsigned long long* hT = hA + (hist_words >= 2u ? hist_words - 2u : 0u);  // LDS_HIST: {T, ambiguous}
    double* hW = reinterpret_cast<double*>(hA + G);  // KM_LOCAL: W
    const uint32_t buf = src.buf_bytes;
    double2* qtab = reinterpret_cast<double2*>(smem + hist_bytes);  // KM_LOCAL only
    double* wtab = reinterpret_cast<double*>(qtab + QLUT_LEN);         // KM_LOCAL: weight of a uniform-q window
    const uint32_t qtab_bytes = MODE == KM_LOCAL ? QTAB_BYTES : 0u;
    // per wave: qualities of two passes [2 x buf] (local mode) | bad-mask words | bit-0 planes | bit-1 planes |
    // quality-change words (local mode)
    const uint32_t mw = mask_words(buf);
    unsigned char* wbase = smem + hist_bytes + qtab_bytes + wid * (buf * (MODE == KM_LOCAL ? 2u : 0u) + 32u * mw);
    unsigned char* qbuf0 = wbase;
    unsigned long long* mbuf = reinterpret_cast<unsigned long long*>(wbase + (MODE == KM_LOCAL ? 2u * buf : 0u));
    unsigned long long* p0buf = mbuf + mw;
    unsigned long long* p1buf = p0buf + mw;
    unsigned long long* dbuf = p1buf + mw;

    if (MODE == KM_LOCAL)
        for (uint32_t i = threadIdx.x; i < QLUT_LEN; i += BLOCK_THREADS) {
            const double lut = src.qlut[2 * i], inv = src.qlut[2 * i + 1];
            qtab[i] = make_double2(lut, inv);
            double x = 1.0;  // the window loop below, for k bases of quality i (fm_scanner.cpp:454)
            for (uint32_t j = 0; j < k; ++j) x = div_rn(x, lut, inv);
            wtab[i] = x;
        }
    if (LDS_HIST)
        for (uint32_t i = threadIdx.x; i < hist_words; i += BLOCK_THREADS) hA[i] = 0ull;
    if (LDS_HIST || MODE == KM_LOCAL) __syncthreads();
    unsigned long long* gU = out_a + 2;

    const uint64_t NWV = (uint64_t)gridDim.x * WAVES_PER_BLOCK;
    const uint64_t gw = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + wid;
    const uint64_t nu = PAIRED ? src.n_units / 2 : src.n_units;
    const uint64_t u0 = nu * gw / NWV, u1 = nu * (gw + 1) / NWV;
    const uint64_t r_end = PAIRED ? 2 * u1 : u1;

    uint32_t t_cnt = 0, amb = 0;
    int cmin = -1, cmax = 0;  // carried unit: its first counted group (-1: none yet), ambiguous so far (0/1)
    uint64_t cunit = ~0ull;
    KtStage<NW> stg;
    auto stage_store = [&](const KtCursor<NW>& cu, unsigned char* qb) {
        uint32_t qprev = 0;
#pragma unroll
        for (int j = 0; j <= NW; ++j)
            kt_stage_chunk<MODE>(src, stg.c[j], stg.q[j], 64u * (uint32_t)j + lane, cu.span, qb, mbuf, p0buf,
                                 p1buf, dbuf, qprev, (uint32_t)j);
        wave_sync();
    };
    // keys of a staged pass (LDS bad mask + bit planes) and their first buckets
    auto make_keys = [&](const KtCursor<NW>& cu, bool (&valid)[NW], uint64_t (&key)[NW], uint32_t (&bk)[NW],
                         bool (&uni)[NW]) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            valid[w] = false;
            key[w] = 0;
            uni[w] = false;
            if (cu.has[w]) {
                const uint32_t off = cu.off[w];
                valid[w] = plane_bits2(mbuf, off, k) == 0;  // no bad base in [off, off + k)
                // quality changes at bases off + 1 .. off + k - 1
                uni[w] = MODE == KM_LOCAL && plane_bits2(dbuf, off + 1u, k - 1u) == 0;
                if (valid[w]) key[w] = plane_bits2(p0buf, off, k) | (plane_bits2(p1buf, off, k) << 32);
            }
            if (CK) {
                bk[w] = valid[w] ? kt8_bucket(key[w], (uint32_t)I.kt_bmask) : 0u;
                key[w] = kt8_ck(key[w], k);  // compared with the low 2k bits of the slots
            } else {
                bk[w] = valid[w] ? (kt_hash(key[w]) & (uint32_t)I.kt_bmask) : 0u;
            }
        }
    };
    auto issue_lookups = [&](const uint32_t (&bk)[NW], u32x4 (&sl)[NW][KT_BSLOTS]) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
#if SPEQ_PROBE_NOLOOKUP  // timing probe only (wrong results): every lookup finds an empty bucket
            for (int j = 0; j < (int)KT_BSLOTS; ++j) sl[w][j] = u32x4{0xFFFFFFFFu, 0xFFFFFFFFu, bk[w], 0u};
#else
            const u32x4* pb = reinterpret_cast<const u32x4*>(I.ktab) + (uint64_t)bk[w] * KT_BSLOTS;
#pragma unroll
            for (int j = 0; j < (int)KT_BSLOTS; ++j) sl[w][j] = pb[j];
#endif
        }
    };

    // Two passes deep: at the top of iteration i, the table lookups of pass i are in flight, the cursor of pass
    // i + 1 is known and its bases are loading (issued before the lookups, so waiting for them does not wait for the
    // lookups), and the offsets of pass i + 2 are loading. Iteration i stages pass i + 1, computes its keys and the
    // cursor of pass i + 2, issues the next loads (lookups of pass i + 1 last), and only then resolves pass i: the
    // lookup latency of pass i is covered by the work on pass i + 1.
    uint64_t r = PAIRED ? 2 * u0 : u0, o = 0;
    uint64_t ob, oe;
    KtCursor<NW> cur;
    for (;;) {
        kt_load_offsets(src, r, r_end, lane, ob, oe);
        cur = kt_cursor<NW>(r, o, r_end, ob, oe, lane, k);
        if (cur.any || r >= r_end) break;
        kt_advance(cur, r_end, r, o);
    }
    uint64_t rn = r_end, on = 0, nb = 0, ne = 0;
    KtCursor<NW> nxt;
    nxt.any = 0u;
    bool valid[NW], uni[NW];
    uint64_t key[NW];
    uint32_t bk[NW];
    u32x4 sl[NW][KT_BSLOTS];
    uint32_t par = 0;  // local mode: qualities of pass i in qbuf0 + par * buf
    if (cur.any) {  // (a wave without windows still reaches the block's final __syncthreads)
        kt_advance(cur, r_end, rn, on);
        kt_load_offsets(src, rn, r_end, lane, nb, ne);
        kt_stage_load(src, cur, cur.s0, lane, stg);
        stage_store(cur, qbuf0);
        make_keys(cur, valid, key, bk, uni);
        for (;;) {  // cursor of pass 1 (serially past units without windows)
            nxt = kt_cursor<NW>(rn, on, r_end, nb, ne, lane, k);
            if (nxt.any || rn >= r_end) break;
            kt_advance(nxt, r_end, rn, on);
            kt_load_offsets(src, rn, r_end, lane, nb, ne);
        }
        kt_advance(nxt, r_end, rn, on);
        kt_load_offsets(src, rn, r_end, lane, nb, ne);
        kt_stage_load(src, nxt, cur.s0, lane, stg);
        issue_lookups(bk, sl);
    }

    while (cur.any) {
        unsigned char* qbuf = qbuf0 + (MODE == KM_LOCAL ? par * buf : 0u);        // pass i
        unsigned char* qbufn = qbuf0 + (MODE == KM_LOCAL ? (par ^ 1u) * buf : 0u);  // pass i + 1
        // ---- stage pass i + 1 (pass i's keys are already computed), its keys and first buckets
        bool valid_n[NW], uni_n[NW];
        uint64_t key_n[NW];
        uint32_t bk_n[NW];
        if (nxt.any) stage_store(nxt, qbufn);
        make_keys(nxt, valid_n, key_n, bk_n, uni_n);
        // ---- cursor of pass i + 2 (its offsets were loaded one pass ago)
        KtCursor<NW> nx2 = kt_cursor<NW>(rn, on, r_end, nb, ne, lane, k);
        const bool skipped = !nx2.any && rn < r_end;  // 64 units without a window (rare): handled below
        kt_advance(nx2, r_end, rn, on);
        // ---- issue: offsets of pass i + 3, bases of pass i + 2, then the lookups of pass i + 1
        kt_load_offsets(src, rn, r_end, lane, nb, ne);
        kt_stage_load(src, nx2, cur.s0, lane, stg);
        u32x4 sl_n[NW][KT_BSLOTS];
        issue_lookups(bk_n, sl_n);

        // ---- resolve the lookups of pass i (rarely a further bucket)
        int which[NW];
        uint32_t ilo[NW], ihi[NW];
        bool pend[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            which[w] = -1;
            ilo[w] = ihi[w] = 0;
            pend[w] = valid[w];
        }
        for (;;) {
            bool more = false;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                if (!pend[w]) continue;
                bool empty = false, found = false;
                if (CK) {
                    // Slots fill a bucket in order (k_ktab_fill8), so the first slot whose key bits match is the
                    // k-mer's or (the all-T k-mer only) the first empty one, and the bucket has an empty slot iff
                    // its last slot is empty: one shift + compare + select per slot.
                    const uint32_t pbits = 64u - 2u * k;
                    uint64_t hitv = ~0ull;
#pragma unroll
                    for (int j = 7; j >= 0; --j) {
                        const uint64_t v = (uint64_t)sl[w][j >> 1][2 * (j & 1)] |
                                           ((uint64_t)sl[w][j >> 1][2 * (j & 1) + 1] << 32);
                        hitv = (v >> pbits) == key[w] ? v : hitv;
                    }
                    found = hitv != ~0ull;
                    empty = sl[w][3][2] == 0xFFFFFFFFu && sl[w][3][3] == 0xFFFFFFFFu;
                    if (found) {
                        const uint64_t pl = hitv & ((1ull << pbits) - 1ull);
                        const bool multi = (pl >> (pbits - 1u)) != 0u;
                        which[w] = multi ? -2 : (int)pl;
                        if (EM && multi) {
                            const uint2 iv = I.kt_multi[pl & ((1ull << (pbits - 1u)) - 1ull)];
                            ilo[w] = iv.x;
                            ihi[w] = iv.y;
                        }
                    }
                } else {
                    const uint32_t kl = (uint32_t)key[w], kh = (uint32_t)(key[w] >> 32);
                    uint32_t lo = 0, info = 0;
                    // key planes are < 2^31, so no key matches an empty slot; slots fill in order (k_ktab_fill),
                    // so the bucket has an empty slot iff its last one is empty
#pragma unroll
                    for (int j = 0; j < (int)KT_BSLOTS; ++j) {
                        const bool hit = sl[w][j][0] == kl && sl[w][j][1] == kh;
                        lo = hit ? sl[w][j][2] : lo;
                        info = hit ? sl[w][j][3] : info;
                        found |= hit;
                    }
                    empty = sl[w][KT_BSLOTS - 1][0] == 0xFFFFFFFFu && sl[w][KT_BSLOTS - 1][1] == 0xFFFFFFFFu;
                    if (found) {
                        const bool multi = (info >> 31) != 0u;
                        which[w] = multi ? -2 : (int)info;
                        ilo[w] = lo;
                        ihi[w] = multi ? lo + (info & 0x7FFFFFFFu) : lo + 1u;
                    }
                }
                pend[w] = !(found || empty);
                more |= pend[w];
            }
            if (!more) break;
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if (pend[w]) {
                    if (CK) bk[w] = bk[w] + 1u == (uint32_t)I.kt_bmask ? 0u : bk[w] + 1u;
                    else bk[w] = (bk[w] + 1u) & (uint32_t)I.kt_bmask;
                    const u32x4* pb = reinterpret_cast<const u32x4*>(I.ktab) + (uint64_t)bk[w] * KT_BSLOTS;
#pragma unroll
                    for (int j = 0; j < (int)KT_BSLOTS; ++j) sl[w][j] = pb[j];
                }
        }

        // ---- tallies of pass i (k_scan step 5)
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            if (!valid[w]) continue;
            ++t_cnt;
            if (EM && which[w] == -2) {
                atomicAdd(&src.em_mult[ilo[w]], 1u);
                src.em_hi[ilo[w]] = ihi[w];
            }
            if (which[w] >= 0) {
                double wgt = 0.0;
                if (MODE == KM_LOCAL) {
                    const unsigned char* qw = qbuf + cur.off[w];
                    if (uni[w]) {
                        wgt = wtab[qw[0]];  // the same k divisions, done once per block
                    } else {
                        double x = 1.0;
                        for (uint32_t i = 0; i < k; ++i) {
                            const double2 t = qtab[qw[i]];
                            x = div_rn(x, t.x, t.y);  // == x / t.x (fm_scanner.cpp:454)
                        }
                        wgt = x;
                    }
                }
                if (LDS_HIST) {
                    atomicAdd(&hA[which[w]], 1ull);
                    if (MODE == KM_LOCAL) atomicAdd(&hW[which[w]], wgt);
                } else {
                    atomicAdd(&gU[which[w]], 1ull);
                    if (MODE == KM_LOCAL) atomicAdd(&out_w[which[w]], wgt);
                }
            }
        }
        // ---- ambiguity (k_scan step 6): per unit, its first counted group and whether another group follows. A
        // wave-uniform loop over the pass's units (in order) with two ballots each replaces the segmented min/max scan.
        {
            uint64_t um = cur.units;
            while (um != 0) {
                const uint32_t i = (uint32_t)__builtin_ctzll(um);
                um &= um - 1;
                const uint64_t unit = PAIRED ? ((cur.r + i) >> 1) : (cur.r + i);
                bool seen = false, differs = false;
                int g = -1;
#pragma unroll
                for (int w = 0; w < NW; ++w) {
                    const bool counted = cur.has[w] != 0u && cur.ri[w] == i && valid[w] && which[w] >= 0;
                    const uint64_t m = __ballot(counted);
                    if (m == 0) continue;
                    if (!seen) g = rli(which[w], (uint32_t)__builtin_ctzll(m));
                    seen = true;
                    differs |= __ballot(counted && which[w] != g) != 0;
                }
                if (unit != cunit) {  // the carried unit is complete
                    if (cunit != ~0ull) amb += cmax;
                    cunit = unit;
                    cmin = seen ? g : -1;  // first counted group of the unit
                    cmax = differs ? 1 : 0;  // ambiguous so far
                } else if (seen) {
                    if (cmin < 0) cmin = g;
                    else if (g != cmin) cmax = 1;
                    if (differs) cmax = 1;
                }
            }
        }
        if (skipped) {  // walk past units without windows (serial loads; rare: 64 units shorter than k)
            for (;;) {
                nx2 = kt_cursor<NW>(rn, on, r_end, nb, ne, lane, k);
                if (nx2.any || rn >= r_end) break;
                kt_advance(nx2, r_end, rn, on);
                kt_load_offsets(src, rn, r_end, lane, nb, ne);
            }
            if (nx2.any) {
                kt_advance(nx2, r_end, rn, on);
                kt_load_offsets(src, rn, r_end, lane, nb, ne);
                kt_stage_load(src, nx2, cur.s0, lane, stg);
            }
        }
        // ---- rotate: pass i + 1 becomes pass i
        cur = nxt;
        nxt = nx2;
        par ^= 1u;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            valid[w] = valid_n[w];
            uni[w] = uni_n[w];
            key[w] = key_n[w];
            bk[w] = bk_n[w];
#pragma unroll
            for (int j = 0; j < (int)KT_BSLOTS; ++j) sl[w][j] = sl_n[w][j];
        }
    }

    if (cunit != ~0ull) amb += (uint32_t)cmax;
    const unsigned long long tsum = wave_sum<unsigned long long>((unsigned long long)t_cnt);
    if (lane == 0) {
        unsigned long long* tgt = LDS_HIST ? hT : out_a;
        if (tsum) atomicAdd(&tgt[0], tsum);
        if (amb) atomicAdd(&tgt[1], (unsigned long long)amb);
    }
    if (LDS_HIST) {
        __syncthreads();
        if (threadIdx.x < 2u) {
            const unsigned long long x = hT[threadIdx.x];
            if (x) atomicAdd(&out_a[threadIdx.x], x);
        }
        for (uint32_t g = threadIdx.x; g < G; g += BLOCK_THREADS) {
            const unsigned long long a = hA[g];
            if (a) atomicAdd(&gU[g], a);
            if (MODE == KM_LOCAL) {
                const double x = hW[g];
                if (x != 0.0) atomicAdd(&out_w[g], x);
            }
        }
    }
}

// ---- k-mer interval table construction (per k, once per replica) ----
// Pass 1: every N-free window of every text inserts its packed k-mer into a set (8-B slots, linear probing, CAS);
// each thread rolls the code over a run of consecutive windows. n_distinct counts the keys inserted.
constexpr uint32_t KT_RUN = 64;
__global__ void k_ktab_keys(const uint8_t* __restrict__ text, const uint64_t* __restrict__ tstart,
                            const uint64_t* __restrict__ cum, uint32_t n_texts, uint64_t total, uint32_t k,
                            unsigned long long* __restrict__ keys, uint64_t smask,
                            unsigned long long* __restrict__ n_distinct) {
    const uint64_t nruns = (total + KT_RUN - 1) / KT_RUN;
    unsigned long long added = 0;
    for (uint64_t run = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; run < nruns;
         run += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f0 = run * KT_RUN, f1 = min(total, f0 + KT_RUN);
        uint32_t t = 0, hi = n_texts;  // largest t with cum[t] <= f0 (that text has windows beyond f0)
        while (hi - t > 1) {
            const uint32_t mid = (t + hi) >> 1;
            if (cum[mid] <= f0) t = mid; else hi = mid;
        }
        uint64_t lo_pl = 0, hi_pl = 0;  // bit planes of the window (bit j = base j)
        uint32_t good = 0;  // consecutive ACGT symbols ending at the window's last base
        bool fresh = true;
        for (uint64_t f = f0; f < f1; ++f) {
            while (f >= cum[t + 1]) {
                ++t;
                fresh = true;
            }
            const uint8_t* base = text + tstart[t] + (f - cum[t]);
            if (fresh) {
                lo_pl = hi_pl = 0;
                good = 0;
                for (uint32_t i = 0; i < k; ++i) {
                    const uint32_t c = base[i];  // SA alphabet: A..T = 2..5, N = 6
                    const bool acgt = c >= 2u && c <= 5u;
                    const uint32_t sym = acgt ? c - 2u : 0u;
                    lo_pl |= (uint64_t)(sym & 1u) << i;
                    hi_pl |= (uint64_t)(sym >> 1) << i;
                    good = acgt ? good + 1u : 0u;
                }
                fresh = false;
            } else {
                const uint32_t c = base[k - 1];
                const bool acgt = c >= 2u && c <= 5u;
                const uint32_t sym = acgt ? c - 2u : 0u;
                lo_pl = (lo_pl >> 1) | ((uint64_t)(sym & 1u) << (k - 1));
                hi_pl = (hi_pl >> 1) | ((uint64_t)(sym >> 1) << (k - 1));
                good = acgt ? good + 1u : 0u;
            }
            const uint64_t code = lo_pl | (hi_pl << 32);
            if (good < k) continue;
            uint64_t sl = kt_hash(code) & smask;  // smask < 2^32
            for (;;) {
                unsigned long long prev = __atomic_load_n(&keys[sl], __ATOMIC_RELAXED);
                if (prev == KT_EMPTY) prev = atomicCAS(&keys[sl], KT_EMPTY, (unsigned long long)code);
                if (prev == KT_EMPTY) {
                    ++added;
                    break;
                }
                if (prev == code) break;
                sl = (sl + 1) & smask;
            }
        }
    }
    if (added) atomicAdd(n_distinct, added);
}

// Pass 2: each distinct k-mer is searched once with the FM-index (search_packed_n: q-mer table + LF steps + run
// classification, exactly as a scan would) and stored with its interval and classification.
__global__ void k_ktab_fill(DevView I, const unsigned long long* __restrict__ keys, uint64_t n_slots, uint32_t k,
                            uint4* __restrict__ table, uint64_t bmask) {
    const Rsrc R = make_rsrc(I);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_slots;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long code = keys[i];
        if (code == KT_EMPTY) continue;
        const uint64_t P[1] = {kt_code(code, k)};
        const bool act[1] = {true};
        int out[1];
        uint32_t lo[1], hi[1];
        search_packed_n<1>(I, R, P, act, k, out, lo, hi);
        if (out[0] == -1) continue;  // unreachable: every key occurs in the texts
        const uint32_t info = out[0] == -2 ? (0x80000000u | (hi[0] - lo[0])) : (uint32_t)out[0];
        uint64_t b = kt_hash(code) & bmask;  // bmask < 2^32
        for (bool placed = false; !placed; b = (b + 1) & bmask) {
            for (uint32_t j = 0; j < KT_BSLOTS && !placed; ++j) {
                uint4* slot = table + b * KT_BSLOTS + j;
                if (atomicCAS(reinterpret_cast<unsigned long long*>(slot), KT_EMPTY, code) == KT_EMPTY) {
                    slot->z = lo[0];
                    slot->w = info;
                    placed = true;
                }
            }
        }
    }
}

// Pass 2 of a compact table (k <= KT8_MAX_K): same search per distinct k-mer; multi-group k-mers get an index into
// `multi` ({lo, hi}, for EM); slots are placed with one 64-bit CAS. n_multi > multi_cap means the payload bits did not
// suffice: the caller builds the 16-B-slot table instead.
__global__ void k_ktab_fill8(DevView I, const unsigned long long* __restrict__ keys, uint64_t n_slots, uint32_t k,
                             unsigned long long* __restrict__ table, uint32_t nb, uint2* __restrict__ multi,
                             unsigned int* __restrict__ n_multi, uint32_t multi_cap) {
    const Rsrc R = make_rsrc(I);
    const uint32_t kb = 2u * k, pbits = 64u - kb;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_slots;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long key = keys[i];
        if (key == KT_EMPTY) continue;
        const uint64_t P[1] = {kt_code(key, k)};
        const bool act[1] = {true};
        int out[1];
        uint32_t lo[1], hi[1];
        search_packed_n<1>(I, R, P, act, k, out, lo, hi);
        if (out[0] == -1) continue;  // unreachable: every key occurs in the texts
        uint64_t pl;
        if (out[0] == -2) {
            const uint32_t m = atomicAdd(n_multi, 1u);
            if (m < multi_cap) multi[m] = make_uint2(lo[0], hi[0]);
            pl = (1ull << (pbits - 1u)) | (uint64_t)(m < multi_cap ? m : 0u);
        } else {
            pl = (uint64_t)out[0];
        }
        const unsigned long long v = (kt8_ck(key, k) << pbits) | pl;
        uint32_t b = kt8_bucket(key, nb);
        for (bool placed = false; !placed; b = (b + 1u == nb) ? 0u : b + 1u)
            for (uint32_t j = 0; j < 8u && !placed; ++j)
                placed = atomicCAS(&table[(uint64_t)b * 8u + j], KT_EMPTY, v) == KT_EMPTY;
    }
}

}  // namespace

namespace {

using namespace speq_dev;


template <int MODE, bool PAIRED, bool LDS, bool KT>
void allow_big_lds_kt() {
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan<MODE, PAIRED, LDS, 1, false, KT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan<MODE, PAIRED, LDS, 2, false, KT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (MODE != KM_REF)
        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan<MODE, PAIRED, LDS, 1, MODE != KM_REF, KT>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (KT && MODE == KM_GLOBAL)
        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan<MODE, PAIRED, LDS, 4, false, KT>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

template <int MODE, bool PAIRED, bool LDS, bool CK>
void allow_big_lds_ktp() {
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_kt<MODE, PAIRED, LDS, false, 1, CK>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_kt<MODE, PAIRED, LDS, false, 2, CK>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_kt<MODE, PAIRED, LDS, true, 1, CK>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

template <int MODE, bool PAIRED, bool LDS>
void allow_big_lds() {
    allow_big_lds_kt<MODE, PAIRED, LDS, false>();
    allow_big_lds_kt<MODE, PAIRED, LDS, true>();
    if constexpr (MODE != KM_REF) {
        allow_big_lds_ktp<MODE, PAIRED, LDS, false>();
        allow_big_lds_ktp<MODE, PAIRED, LDS, true>();
    }
}

void allow_big_lds_all() {
    allow_big_lds<KM_GLOBAL, false, true>();
    allow_big_lds<KM_GLOBAL, false, false>();
    allow_big_lds<KM_GLOBAL, true, true>();
    allow_big_lds<KM_GLOBAL, true, false>();
    allow_big_lds<KM_LOCAL, false, true>();
    allow_big_lds<KM_LOCAL, false, false>();
    allow_big_lds<KM_LOCAL, true, true>();
    allow_big_lds<KM_LOCAL, true, false>();
    allow_big_lds<KM_REF, false, true>();
    allow_big_lds<KM_REF, false, false>();
}

// The q-mer table level for a scan of k-mers: the longest of q, q-1, q-2 that leaves a number of symbols divisible
// by the widest LF step (3 with occ3, 2 with occ2), so the search needs no leftover single/pair step; any level
// gives the same intervals (tests/test_gpu_parity.py runs each).
// The sparse forms of the q-mer tables (tuning "sparse_prefix" 1 or -1): per level a rank directory of 96 codes per
// entry over the codes that occur, and their intervals. Built from the dense tables on the first tuning that asks for
// them (a host pass over 4^q codes, 50 ms at q = 12, that every device open paid until round 6; the default dense
// lookups never read them).
void build_sparse(speq_device_index* d) {
    std::lock_guard<std::mutex> lk(d->sparse_mu);
    if (d->sparse_built) return;
    DeviceGuard g(d->device);
    for (int lvl = 0; lvl < 3; ++lvl) {
        if (d->prefix_level[lvl] == nullptr || d->prefix_words[lvl] == 0) continue;
        std::vector<uint32_t> t(d->prefix_words[lvl]);
        HIP_OK(hipMemcpy(t.data(), d->prefix_level[lvl], t.size() * 4, hipMemcpyDeviceToHost));
        const uint64_t Q = t.size() / 2, nbk = Q / 96 + 1;
        std::vector<speq::OccEntry> rk(nbk, speq::OccEntry{});
        std::vector<uint32_t> iv;
        uint32_t cnt = 0;
        for (uint64_t c = 0; c < Q; ++c) {
            if (c % 96 == 0) rk[c / 96].count = cnt;
            if (t[2 * c] < t[2 * c + 1]) {
                rk[c / 96].bits[(c % 96) / 32] |= 1u << (c % 32);
                iv.push_back(t[2 * c]);
                iv.push_back(t[2 * c + 1]);
                ++cnt;
            }
        }
        if (Q % 96 == 0) rk[nbk - 1].count = cnt;
        d->present[lvl] = cnt;
        if (iv.empty()) iv.assign(2, 0u);
        d->sparse_rank[lvl] = reinterpret_cast<const uint4*>(d->track(dev_upload(rk)));
        d->sparse_iv[lvl] = reinterpret_cast<const uint2*>(d->track(dev_upload(iv)));
    }
    d->sparse_built = true;
}

void use_sparse(const speq_device_index* d, uint32_t lvl, DevView& v) {
    v.pfx_rank = nullptr;
    v.pfx_iv = nullptr;
    if (d->sparse_rank[lvl] == nullptr) return;
    const uint64_t codes = uint64_t(1) << (2 * (d->base_q - lvl));
    const bool sparse = d->sparse_choice == 1 || (d->sparse_choice < 0 && d->present[lvl] * 8 < codes);
    if (sparse) {
        v.pfx_rank = d->sparse_rank[lvl];
        v.pfx_iv = d->sparse_iv[lvl];
    }
}

DevView view_for_k(const speq_device_index* d, uint32_t k) {
    DevView v = d->view;
    const uint32_t q = d->base_q;
    if (q == 0 || k < 1) return v;
    const uint32_t step = v.occ3 ? 3u : (v.occ2 ? 2u : 1u);
    for (uint32_t lvl = 0; lvl < 3; ++lvl) {
        if (lvl >= q || d->prefix_level[lvl] == nullptr) break;
        const uint32_t qq = q - lvl;
        if (qq <= k && (k - qq) % step == 0) {
            v.q = qq;
            v.prefix = d->prefix_level[lvl];
            use_sparse(d, lvl, v);
            return v;
        }
    }
    use_sparse(d, 0, v);
    return v;
}

// The index view a scan of k-mers uses (q-mer table level by k unless forced), without the k-mer table.
DevView scan_view(const speq_device_index* d, uint32_t k) {
    DevView v = d->view;
    if (d->prefix_choice >= 0) use_sparse(d, (uint32_t)d->prefix_choice, v);
    else v = view_for_k(d, k);
    v.ktab = nullptr;
    v.kt_bmask = 0;
    v.kt_k = 0;
    return v;
}

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Builds the k-mer interval table of k on the replica's stream (blocking): the distinct N-free k-mers of the texts
// (k_ktab_keys into a set of 2x the window count), then one FM-index search per distinct k-mer (k_ktab_fill) into
// buckets sized for a load factor in (1/4, 1/2].
speq_device_index::KmerTable build_ktab(speq_device_index* d, uint32_t k) {
    DeviceGuard g(d->device);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint64_t> cum(d->n_texts + 1, 0);
    for (uint32_t t = 0; t < d->n_texts; ++t) {
        const uint64_t L = d->text_start[t + 1] - d->text_start[t] - 1;
        cum[t + 1] = cum[t] + (L >= k ? L - k + 1 : 0);
    }
    const uint64_t total = cum[d->n_texts];
    speq_device_index::KmerTable kt;
    void* keys = nullptr;
    uint64_t* d_cum = nullptr;
    unsigned long long* d_cnt = nullptr;
    void* tab = nullptr;       // compact-table build: freed here unless handed to the replica
    uint2* multi = nullptr;
    unsigned int* d_nm = nullptr;
    auto cleanup = [&] {
        (void)hipStreamSynchronize(d->stream);
        if (keys) (void)hipFree(keys);
        if (d_cum) (void)hipFree(d_cum);
        if (d_cnt) (void)hipFree(d_cnt);
        if (tab) (void)hipFree(tab);
        if (multi) (void)hipFree(multi);
        if (d_nm) (void)hipFree(d_nm);
        keys = nullptr;
        d_cum = nullptr;
        d_cnt = nullptr;
        tab = nullptr;
        multi = nullptr;
        d_nm = nullptr;
    };
    try {
        unsigned long long distinct = 0;
        const uint64_t slots = next_pow2(std::max<uint64_t>(2 * total, 64));
        // too large for 32-bit bucket hashing, or for the free HBM (key set + a table of up to 4 slots per window):
        // no table, scans of this k use LF steps (same results)
        size_t free_b = 0, total_b = 0;
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        const uint64_t need = slots * 8 + next_pow2(std::max<uint64_t>(1, total * d->kt_slots / KT_BSLOTS)) * 16 * KT_BSLOTS;
        if (slots > (1ull << 32) || need > free_b / 10 * 9) return kt;  // kt.table == nullptr
        if (total > 0) {
            HIP_OK(hipMalloc(&keys, slots * 8));
            HIP_OK(hipMalloc(&d_cum, cum.size() * 8));
            HIP_OK(hipMalloc(&d_cnt, 8));
            HIP_OK(hipMemsetAsync(keys, 0xFF, slots * 8, d->stream));
            HIP_OK(hipMemsetAsync(d_cnt, 0, 8, d->stream));
            HIP_OK(hipMemcpyAsync(d_cum, cum.data(), cum.size() * 8, hipMemcpyHostToDevice, d->stream));
            const uint64_t runs = (total + KT_RUN - 1) / KT_RUN;
            const uint32_t grid = (uint32_t)std::min<uint64_t>((runs + 255) / 256, 8192);
            hipLaunchKernelGGL(k_ktab_keys, dim3(grid), dim3(256), 0, d->stream, d->d_text, d->d_text_start, d_cum,
                               d->n_texts, total, k, reinterpret_cast<unsigned long long*>(keys), slots - 1, d_cnt);
            HIP_OK(hipGetLastError());
            HIP_OK(hipMemcpyAsync(&distinct, d_cnt, 8, hipMemcpyDeviceToHost, d->stream));
            HIP_OK(hipStreamSynchronize(d->stream));
        }
        kt.distinct = distinct;
        // compact form first (k <= KT8_MAX_K): sized for the load factor kt_load8; if the multi-group k-mers outgrow the
        // payload bits, fall through to the 16-B-slot form
        const uint32_t pbits = 64u - 2u * k;
        const uint64_t multi_cap = std::min<uint64_t>(distinct, (1ull << (pbits - 1u)) - 2u);
        const uint64_t nb8 = std::max<uint64_t>(1, (uint64_t)((double)distinct * 100.0 / (8.0 * d->kt_load8)) + 1);
        // the fill writes the multi-group k-mers into a scratch array of the worst-case size (every distinct k-mer),
        // copied to one of the exact size afterwards; the free-memory check covers the scratch
        const bool try_compact = d->kt_compact && KT_BSLOTS == 4 && k <= KT8_MAX_K && distinct > 0 && nb8 < (1ull << 32);
        if (try_compact && nb8 * 64 + std::max<uint64_t>(multi_cap, 1) * 8 > free_b / 10 * 9) {
            cleanup();
            return kt;  // kt.table == nullptr: LF steps
        }
        if (try_compact) {
            HIP_OK(hipMalloc(&tab, nb8 * 64));
            HIP_OK(hipMalloc(&multi, std::max<uint64_t>(multi_cap, 1) * 8));
            HIP_OK(hipMalloc(&d_nm, 4));
            HIP_OK(hipMemsetAsync(tab, 0xFF, nb8 * 64, d->stream));
            HIP_OK(hipMemsetAsync(d_nm, 0, 4, d->stream));
            const DevView v = scan_view(d, k);
            const uint32_t grid = (uint32_t)std::min<uint64_t>((slots + 255) / 256, 16384);
            hipLaunchKernelGGL(k_ktab_fill8, dim3(grid), dim3(256), 0, d->stream, v,
                               reinterpret_cast<const unsigned long long*>(keys), slots, k,
                               reinterpret_cast<unsigned long long*>(tab), (uint32_t)nb8, multi, d_nm,
                               (uint32_t)multi_cap);
            HIP_OK(hipGetLastError());
            unsigned int n_multi = 0;
            HIP_OK(hipMemcpyAsync(&n_multi, d_nm, 4, hipMemcpyDeviceToHost, d->stream));
            HIP_OK(hipStreamSynchronize(d->stream));
            if (n_multi <= multi_cap) {
                uint2* exact = nullptr;
                HIP_OK(hipMalloc(&exact, std::max<uint64_t>(n_multi, 1) * 8));
                if (n_multi)
                    HIP_OK(hipMemcpyAsync(exact, multi, (uint64_t)n_multi * 8, hipMemcpyDeviceToDevice, d->stream));
                HIP_OK(hipStreamSynchronize(d->stream));
                kt.compact = true;
                kt.table = reinterpret_cast<uint4*>(d->track(tab));
                kt.multi = d->track(exact);
                kt.buckets = nb8;
                kt.bytes = nb8 * 64 + std::max<uint64_t>(n_multi, 1) * 8;  // what the replica keeps
                tab = nullptr;  // owned by the replica now
                cleanup();
                kt.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                return kt;
            }
            (void)hipFree(tab);
            (void)hipFree(multi);
            (void)hipFree(d_nm);
            tab = nullptr;
            multi = nullptr;
            d_nm = nullptr;
        }
        kt.buckets = next_pow2(std::max<uint64_t>(1, (distinct * d->kt_slots + KT_BSLOTS - 1) / KT_BSLOTS));
        kt.bytes = kt.buckets * 16 * KT_BSLOTS;
        HIP_OK(hipMalloc(&kt.table, kt.buckets * 16 * KT_BSLOTS));
        d->track(kt.table);
        HIP_OK(hipMemsetAsync(kt.table, 0xFF, kt.buckets * 16 * KT_BSLOTS, d->stream));
        if (distinct > 0) {
            const DevView v = scan_view(d, k);
            const uint32_t grid = (uint32_t)std::min<uint64_t>((slots + 255) / 256, 16384);
            hipLaunchKernelGGL(k_ktab_fill, dim3(grid), dim3(256), 0, d->stream, v,
                               reinterpret_cast<const unsigned long long*>(keys), slots, k, kt.table, kt.buckets - 1);
            HIP_OK(hipGetLastError());
        }
        HIP_OK(hipStreamSynchronize(d->stream));
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
    kt.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return kt;
}

// The table of k (built on first use), or null when tables are off or k is outside 1..31.
const speq_device_index::KmerTable* ensure_ktab(speq_device_index* d, uint32_t k) {
    if (!d->kmer_table || k < 1 || k > KT_MAX_K) return nullptr;
    std::lock_guard<std::mutex> lk(d->kt_mu);
    auto it = d->ktabs.find(k);
    if (it == d->ktabs.end()) it = d->ktabs.emplace(k, build_ktab(d, k)).first;
    return it->second.table ? &it->second : nullptr;  // null table: too large, LF steps
}

template <int MODE, bool PAIRED, bool LDS, bool CK>
void launch_kt(const DevView& v, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st, unsigned long long* a,
               double* w, uint32_t ilp) {
    if (src.em_mult != nullptr)
        hipLaunchKernelGGL((k_scan_kt<MODE, PAIRED, LDS, true, 1, CK>), dim3(grid), dim3(BLOCK_THREADS), lds, st, v,
                           src, a, w);
    else if (ilp == 2)
        hipLaunchKernelGGL((k_scan_kt<MODE, PAIRED, LDS, false, 2, CK>), dim3(grid), dim3(BLOCK_THREADS), lds, st, v,
                           src, a, w);
    else
        hipLaunchKernelGGL((k_scan_kt<MODE, PAIRED, LDS, false, 1, CK>), dim3(grid), dim3(BLOCK_THREADS), lds, st, v,
                           src, a, w);
}

template <int MODE, bool PAIRED, bool LDS, bool KT>
void launch_v(const speq_device_index* d, const DevView& v, const UnitSrc& src, uint32_t grid, size_t lds,
              hipStream_t st, unsigned long long* a, unsigned long long* b, double* w) {
    const uint32_t ilp = KT ? (d->ilp_kt ? d->ilp_kt : (v.kt_compact ? 1u : 2u))
                            : (MODE == KM_LOCAL ? d->ilp_local : d->ilp);
    if constexpr (KT && MODE != KM_REF) {
        if (ilp <= 2 && d->kt_pipeline) {  // software-pipelined table scan
            if (v.kt_compact) launch_kt<MODE, PAIRED, LDS, true>(v, src, grid, lds, st, a, w, ilp);
            else launch_kt<MODE, PAIRED, LDS, false>(v, src, grid, lds, st, a, w, ilp);
            return;
        }
    }
    if (MODE != KM_REF && src.em_mult != nullptr)
        hipLaunchKernelGGL((k_scan<MODE, PAIRED, LDS, 1, MODE != KM_REF, KT>), dim3(grid), dim3(BLOCK_THREADS), lds,
                           st, v, src, a, b, w);
    else if (KT && MODE == KM_GLOBAL && ilp == 4)
        hipLaunchKernelGGL((k_scan<MODE, PAIRED, LDS, 4, false, KT>), dim3(grid), dim3(BLOCK_THREADS), lds, st, v,
                           src, a, b, w);
    else if (ilp >= 2)
        hipLaunchKernelGGL((k_scan<MODE, PAIRED, LDS, 2, false, KT>), dim3(grid), dim3(BLOCK_THREADS), lds, st, v,
                           src, a, b, w);
    else
        hipLaunchKernelGGL((k_scan<MODE, PAIRED, LDS, 1, false, KT>), dim3(grid), dim3(BLOCK_THREADS), lds, st, v,
                           src, a, b, w);
}

template <int MODE, bool PAIRED, bool LDS>
void launch_t(const speq_device_index* d, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
              unsigned long long* a, unsigned long long* b, double* w, const speq_device_index::KmerTable* kt) {
    DevView v = scan_view(d, src.k);
    // a compact table is read only by the pipelined table kernel; other scans of this k take LF steps
    if (kt && kt->compact && !(MODE != KM_REF && d->ilp_kt <= 2 && d->kt_pipeline))
        kt = nullptr;
    if (kt) {
        v.ktab = kt->table;
        v.kt_bmask = kt->compact ? kt->buckets : kt->buckets - 1;
        v.kt_multi = kt->multi;
        v.kt_compact = kt->compact ? 1u : 0u;
        v.kt_k = src.k;
    }
    if (MODE != KM_REF)
        const_cast<speq_device_index*>(d)->last_kernel =
            kt ? ((d->ilp_kt <= 2 && d->kt_pipeline) || kt->compact ? 2 : 1) : 0;
    if (kt) launch_v<MODE, PAIRED, LDS, true>(d, v, src, grid, lds, st, a, b, w);
    else launch_v<MODE, PAIRED, LDS, false>(d, v, src, grid, lds, st, a, b, w);
}

// returns the kernel it launched (speq_device_get_tuning "last_kernel" codes: 0 LF steps, 1/2 k-mer table, 3 ax)
int launch_scan(speq_device_index* d, int mode, bool paired, const UnitSrc& src, uint64_t work_units,
                hipStream_t st, unsigned long long* a, unsigned long long* b, double* w) {
    // read scans: the anchor-and-extend kernel when the replica has (or can build) its structures for k (ax_scan.hip)
    if (mode != KM_REF && speq::launch_ax(d, mode, paired, src, st, a, w)) {
        d->last_kernel = 3;
        return 3;
    }
    if (src.ax_stats) return -1;  // the diagnostic twin exists for k_scan_ax only: launch nothing
    const speq_device_index::KmerTable* kt = ensure_ktab(d, src.k);
    const bool lds_hist = d->G <= LDS_HIST_MAX_G;
    const uint32_t hist_words = lds_hist ? ((mode == KM_GLOBAL) ? d->G : 2u * d->G) + 2u : 0u;
    const size_t lds = ((hist_words * 8u + 15u) & ~15u) + (mode == KM_LOCAL ? QTAB_BYTES : 0u) +
                       (size_t)WAVES_PER_BLOCK * wave_lds_bytes(src.buf_bytes, mode == KM_LOCAL);
    // >= 4 units (or 256 windows) per wave; grid capped (default 4096 = 2x the 8 resident blocks x 256 CUs).
    uint64_t blocks = (work_units + 4 * WAVES_PER_BLOCK - 1) / (4 * WAVES_PER_BLOCK);
    if (blocks < 1) blocks = 1;
    const uint32_t grid_cap = kt ? d->grid_blocks_kt : d->grid_blocks;
    if (blocks > grid_cap) blocks = grid_cap;
    size_t lds_launch = lds;
    const uint32_t bpc = kt ? d->blocks_per_cu_kt : d->blocks_per_cu;
    if (bpc > 0) {  // occupancy cap: pad dynamic LDS so only bpc blocks fit a CU
        const size_t pad = (160u * 1024u) / bpc;
        if (pad > lds_launch) lds_launch = pad & ~(size_t)15;
    }
    const uint32_t grid = (uint32_t)blocks;
#define SPEQ_DISPATCH(M, P)                                                            \
    do {                                                                               \
        if (lds_hist) launch_t<M, P, true>(d, src, grid, lds_launch, st, a, b, w, kt); \
        else launch_t<M, P, false>(d, src, grid, lds_launch, st, a, b, w, kt);         \
    } while (0)
    if (mode == KM_REF) SPEQ_DISPATCH(KM_REF, false);
    else if (mode == KM_GLOBAL) { if (paired) SPEQ_DISPATCH(KM_GLOBAL, true); else SPEQ_DISPATCH(KM_GLOBAL, false); }
    else { if (paired) SPEQ_DISPATCH(KM_LOCAL, true); else SPEQ_DISPATCH(KM_LOCAL, false); }
#undef SPEQ_DISPATCH
    HIP_OK(hipGetLastError());
    return kt ? ((d->ilp_kt <= 2 && d->kt_pipeline) || kt->compact ? 2 : 1) : 0;
}

}  // namespace

namespace speq {
DevView search_view(const speq_device_index* d, uint32_t k) { return scan_view(d, k); }
}  // namespace speq

// ---- scan implementations shared by the plain and the EM-histogram entry points ----
// returns the kernel it launched (launch_scan), -1 with ax_stats when k_scan_ax cannot take the scan (nothing launched)
static int scan_device_impl(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual, const uint64_t* d_offsets,
                      uint64_t n_reads, const speq_scan_params* p, uint64_t* d_counts, double* d_weights,
                      uint32_t* em_mult, uint32_t* em_hi, hipStream_t st, unsigned long long* ax_stats = nullptr) {
    if (!d || !p || !d_counts) throw std::invalid_argument("speq_scan_reads_device: null argument");
    if (p->k < 1 || p->k > MAX_K) throw std::invalid_argument("speq_scan_reads_device: k must be in [1, 4096]");
    if (p->mode != SPEQ_MODE_GLOBAL && p->mode != SPEQ_MODE_LOCAL)
        throw std::invalid_argument("speq_scan_reads_device: bad mode");
    if (p->mode == SPEQ_MODE_LOCAL && !d_weights)
        throw std::invalid_argument("speq_scan_reads_device: local mode needs a weights buffer");
    if (p->paired && (n_reads & 1)) throw std::invalid_argument("speq_scan_reads_device: paired scan needs an even record count");
    if (n_reads == 0) return ax_stats ? -1 : 0;
    if (!d_seq || !d_qual || !d_offsets) throw std::invalid_argument("speq_scan_reads_device: null read buffer");
    DeviceGuard g(d->device);
    UnitSrc src{};
    src.seq = d_seq;
    src.qual = d_qual;
    src.off = d_offsets;
    src.qlut = d->d_qlut;
    src.em_mult = em_mult;
    src.em_hi = em_hi;
    src.n_units = n_reads;
    src.end_adj = 0;
    src.k = p->k;
    src.cutoff = p->phred_cutoff;
    src.buf_bytes = staging_bytes(p->k, std::max({d->ilp, d->ilp_local, d->ilp_kt ? d->ilp_kt : 2u}));
    src.ax_stats = ax_stats;
    const int mode = p->mode == SPEQ_MODE_LOCAL ? KM_LOCAL : KM_GLOBAL;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->timing) {
        HIP_OK(hipEventCreate(&e0));
        HIP_OK(hipEventCreate(&e1));
        HIP_OK(hipEventRecord(e0, st));
    }
    const int kernel = launch_scan(d, mode, p->paired != 0, src, p->paired ? n_reads / 2 : n_reads, st,
                                   reinterpret_cast<unsigned long long*>(d_counts), nullptr, d_weights);
    if (d->timing) {
        if (kernel < 0) {  // nothing was launched (ax_stats, the anchor kernel cannot take it): no interval to time
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            return kernel;
        }
        HIP_OK(hipEventRecord(e1, st));
        std::lock_guard<std::mutex> lk(d->events_mu);
        d->events.emplace_back(e0, e1);
    }
    return kernel;
}


// dst += src for the EM interval histogram; an interval's end is a function of its start, so a start that src
// recorded takes src's end (dst's is either the same or unset). Grid-stride loop.
// EM finalize: the positions that start a recorded interval, compacted in position order (the CSR rows keep the
// order the host built before, so the EM step's sums are unchanged). Block b covers EM_TILE positions; pass 1 counts
// them, an exclusive scan of the counts (one workgroup) gives every block its offset, pass 2 writes (lo, mult, hi).
constexpr uint32_t EM_TILE = 4096;
__global__ __launch_bounds__(256) void k_em_count(const uint32_t* __restrict__ mult, uint64_t n,
                                                  uint32_t* __restrict__ counts) {
    __shared__ uint32_t part[4];
    const uint64_t b0 = (uint64_t)blockIdx.x * EM_TILE;
    uint32_t c = 0;
    for (uint32_t i = threadIdx.x; i < EM_TILE; i += 256) {
        const uint64_t pos = b0 + i;
        c += (pos < n && mult[pos] != 0u) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
    if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}
// exclusive scan of nb block counts in place, one workgroup of 1024 threads; total at counts[nb]
__global__ __launch_bounds__(1024) void k_em_scan(uint32_t* __restrict__ counts, uint32_t nb) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nb ? counts[i] : 0u;
        uint32_t x = v;  // inclusive scan within the wave
        const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t before = carry;
        for (uint32_t q = 0; q < w; ++q) before += wsum[q];
        if (i < nb) counts[i] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[nb] = carry;
}
__global__ __launch_bounds__(256) void k_em_compact(const uint32_t* __restrict__ mult, const uint32_t* __restrict__ hi,
                                                    uint64_t n, const uint32_t* __restrict__ offs,
                                                    uint32_t* __restrict__ out_lo, uint32_t* __restrict__ out_mult,
                                                    uint32_t* __restrict__ out_hi) {
    __shared__ uint32_t wtot[4];
    __shared__ uint32_t run;
    const uint64_t b0 = (uint64_t)blockIdx.x * EM_TILE;
    if (threadIdx.x == 0) run = offs[blockIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    for (uint32_t i = 0; i < EM_TILE; i += 256) {  // 256 consecutive positions per round, in order
        const uint64_t pos = b0 + i + threadIdx.x;
        const uint32_t m = pos < n ? mult[pos] : 0u;
        const unsigned long long bal = __ballot(m != 0u);
        if (lane == 0) wtot[w] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t at = run;
        for (uint32_t q = 0; q < w; ++q) at += wtot[q];
        if (m != 0u) {
            at += __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            out_lo[at] = (uint32_t)pos;
            out_mult[at] = m;
            out_hi[at] = hi[pos];
        }
        __syncthreads();
        if (threadIdx.x == 0) run += wtot[0] + wtot[1] + wtot[2] + wtot[3];
        __syncthreads();
    }
}

__global__ void k_em_merge(uint32_t* __restrict__ dmult, uint32_t* __restrict__ dhi, const uint32_t* __restrict__ smult,
                           const uint32_t* __restrict__ shi, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t m = smult[i];
        if (m) {
            dmult[i] += m;
            dhi[i] = shi[i];
        }
    }
}

extern "C" {

int speq_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int speq_device_open(const speq_index* idx, int device, speq_device_index** out) {
    return speq::guarded([&] {
        if (!idx || !out) throw std::invalid_argument("speq_device_open: null argument");
        int ndev = speq_device_count();
        if (ndev <= 0) throw speq::DeviceError("no GPU visible (the scan path has no CPU fallback)");
        if (device < 0 || device >= ndev) throw std::invalid_argument("speq_device_open: bad device ordinal");
        DeviceGuard g(device);
        speq::startup_trace("device open: start");
        const speq::FmIndex& fm = idx->fm;
        auto d = std::make_unique<speq_device_index>();
        d->device = device;
        d->G = fm.n_groups;
        d->n_texts = fm.n_texts;
        d->text_start = fm.text_start;
        DevView& v = d->view;
        v.occ = reinterpret_cast<const uint4*>(d->track(dev_upload(fm.occ)));
        v.nb = (uint32_t)fm.n_blocks();
        v.occ2 = reinterpret_cast<const uint4*>(d->track(dev_upload(fm.occ2)));
        v.occ3 = reinterpret_cast<const uint4*>(d->track(dev_upload(fm.occ3)));
        v.runs = reinterpret_cast<const uint4*>(d->track(dev_upload(fm.runs)));
        v.run_label = d->track(dev_upload(fm.run_label));
        v.lab = d->track(dev_upload(fm.lab));
        v.prefix = reinterpret_cast<const uint2*>(d->track(dev_upload(fm.prefix)));
        d->prefix_level[0] = v.prefix;
        d->prefix_level[1] = reinterpret_cast<const uint2*>(d->track(dev_upload(fm.prefix1)));
        d->prefix_level[2] = reinterpret_cast<const uint2*>(d->track(dev_upload(fm.prefix2)));
        for (int lvl = 0; lvl < 3; ++lvl)  // (the sparse forms are built on first use: build_sparse)
            d->prefix_words[lvl] = (lvl == 0 ? fm.prefix : lvl == 1 ? fm.prefix1 : fm.prefix2).size();
        speq::startup_trace("device open: FM arrays");
        v.n = (uint32_t)fm.n;
        v.q = fm.prefix_q;
        d->base_q = fm.prefix_q;
        v.G = fm.n_groups;
        d->d_text = d->track(dev_upload(fm.text));
        d->d_text_start = d->track(dev_upload(fm.text_start));
        d->d_text_group = d->track(dev_upload(fm.text_group));
        std::vector<double> lut(2 * QLUT_LEN);  // {1 - 1/10^(q/10) (fm_scanner.cpp:454), its reciprocal}
        for (uint32_t q = 0; q < QLUT_LEN; ++q) {
            lut[2 * q] = 1.0 - 1.0 / std::pow(10.0, (double)q / 10.0);
            lut[2 * q + 1] = 1.0 / lut[2 * q];  // q = 0: inf, never used (a passing window has every q > cutoff >= 0)
        }
        d->d_qlut = d->track(dev_upload(lut));
        speq::startup_trace("device open: uploads");
        d->stream = static_cast<hipStream_t>(speq::pooled_stream(device));
        hipDeviceProp_t prop;
        HIP_OK(hipGetDeviceProperties(&prop, device));
        d->n_cus = (uint32_t)prop.multiProcessorCount;
        // Default launch shape (measured, profiles/r01/sweep_tuning.jsonl): an index whose ACGT occ planes exceed
        // one XCD's 4 MiB L2 is served from the Infinity Cache, where 3 resident blocks per CU beat full occupancy
        // (fewer concurrent gathers thrashing L1/L2); an L2-resident index wants every wave it can get.
        // (With the two-symbol planes the gather chain is half as long and full occupancy wins again.)
        const uint64_t acgt_bytes = 4ull * fm.n_blocks() * sizeof(speq::OccEntry);
        d->blocks_per_cu = (fm.occ2.empty() && acgt_bytes > (4ull << 20)) ? 3u : 0u;
        if (!fm.occ3.empty()) {
            // With the three-symbol planes (measured, profiles/r01/sweep_grid_triples.jsonl, sweep_bpc_cfg*.jsonl):
            // planes that spill L2 but fit the 256 MB Infinity Cache want 4 blocks/CU (cfg 3: +12 %); planes that
            // spill the Infinity Cache too, so gathers go to HBM, want 3 (cfg 5: 2.1x); small ones want them all.
            const uint64_t plane_bytes = (fm.occ.size() + fm.occ2.size() + fm.occ3.size()) * sizeof(speq::OccEntry);
            d->blocks_per_cu = plane_bytes <= (16ull << 20) ? 0u : (plane_bytes <= (256ull << 20) ? 4u : 3u);
        }
        d->grid_blocks = fm.n < (4ull << 20) ? 16384u : 8192u;
        // Two windows per lane pay off on small (L2/MALL-hot) indexes (cfg 2, n = 1 M: +3 %); on larger ones the
        // extra gathers in flight thrash the caches (cfg 3, n = 10 M: -15 %). profiles/r01/ab_occupancy.txt,
        // sweep_triples.jsonl
        d->ilp = fm.n < (4ull << 20) ? 2u : 1u;
        allow_big_lds_all();
        speq::startup_trace("device open: end");
        *out = d.release();
    });
}

speq_device_index::~speq_device_index() {
    int prev = -1;
    const bool switched = hipGetDevice(&prev) == hipSuccess && prev != device && hipSetDevice(device) == hipSuccess;
    for (auto& e : events) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    for (void* p : allocs) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
    if (switched) (void)hipSetDevice(prev);
}

int speq_device_close(speq_device_index* d) {
    return speq::guarded([&] {
        if (!d) return;
        speq::release_host_pipelines(d);
        delete d;
    });
}

int speq_scan_reads_device(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual,
                           const uint64_t* d_offsets, uint64_t n_reads, const speq_scan_params* p,
                           uint64_t* d_counts, double* d_weights, void* stream) {
    return speq::guarded([&] {
        scan_device_impl(d, d_seq, d_qual, d_offsets, n_reads, p, d_counts, d_weights, nullptr, nullptr,
                         static_cast<hipStream_t>(stream));
    });
}

int speq_scan_reads_device_stats(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual,
                                 const uint64_t* d_offsets, uint64_t n_reads, const speq_scan_params* p,
                                 uint64_t* d_counts, double* d_weights, uint64_t* stats) {
    return speq::guarded([&] {
        if (!d || !stats) throw std::invalid_argument("speq_scan_reads_device_stats: null argument");
        DeviceGuard g(d->device);
        // the counters' buffer travels with this launch only (UnitSrc::ax_stats), so ordinary scans of the same
        // replica from other threads never run the instrumented kernel
        unsigned long long* ds = nullptr;
        HIP_OK(hipMalloc(&ds, SPEQ_AX_STATS_N * 8));
        struct Release {
            unsigned long long*& p;
            ~Release() {
                if (p) (void)hipFree(p);
            }
        } release{ds};
        HIP_OK(hipMemsetAsync(ds, 0, SPEQ_AX_STATS_N * 8, d->stream));
        HIP_OK(hipStreamSynchronize(d->stream));
        const int kernel =
            scan_device_impl(d, d_seq, d_qual, d_offsets, n_reads, p, d_counts, d_weights, nullptr, nullptr, d->stream, ds);
        if (kernel != 3)
            throw std::invalid_argument("speq_scan_reads_device_stats: the scan did not use the anchor-and-extend kernel");
        HIP_OK(hipStreamSynchronize(d->stream));
        HIP_OK(hipMemcpy(stats, ds, SPEQ_AX_STATS_N * 8, hipMemcpyDeviceToHost));
    });
}

int speq_scan_reads(speq_device_index* d, const uint8_t* seq, const uint8_t* qual, const uint64_t* offsets,
                    uint64_t n_reads, const speq_scan_params* p, uint64_t* counts, double* weights) {
    return speq::guarded([&] { speq::scan_host_pipelined(d, seq, qual, offsets, n_reads, p, nullptr, counts, weights); });
}

// ---- EM histogram (see em.hpp) ----
int speq_em_create(const speq_index* idx, speq_device_index* d, speq_em** out) {
    return speq::guarded([&] {
        if (!idx || !d || !out) throw std::invalid_argument("speq_em_create: null argument");
        if (idx->fm.n != d->view.n) throw std::invalid_argument("speq_em_create: index and device replica differ");
        DeviceGuard g(d->device);
        auto em = std::make_unique<speq_em>();
        em->idx = idx;
        em->dev = d;
        em->n = idx->fm.n;
        em->G = idx->fm.n_groups;
        HIP_OK(hipMalloc(&em->d_mult, em->n * 4));
        HIP_OK(hipMalloc(&em->d_hi, em->n * 4));
        HIP_OK(hipMemset(em->d_mult, 0, em->n * 4));
        // interval ends are merged across ranks / replicas with a max (speq_em_allreduce, k_em_merge): a position this
        // replica never wrote must hold 0, not whatever the allocation held
        HIP_OK(hipMemset(em->d_hi, 0, em->n * 4));
        *out = em.release();
    });
}

int speq_em_scan_reads(speq_em* em, const uint8_t* seq, const uint8_t* qual, const uint64_t* offsets, uint64_t n_reads,
                       const speq_scan_params* p, uint64_t* counts, double* weights) {
    return speq::guarded([&] {
        if (!em || em->finalized) throw std::invalid_argument("speq_em_scan_reads: bad or finalized histogram");
        speq::scan_host_pipelined(em->dev, seq, qual, offsets, n_reads, p, em, counts, weights);
    });
}

int speq_em_scan_reads_device(speq_em* em, const uint8_t* d_seq, const uint8_t* d_qual, const uint64_t* d_offsets,
                              uint64_t n_reads, const speq_scan_params* p, uint64_t* d_counts, double* d_weights,
                              void* stream) {
    return speq::guarded([&] {
        if (!em || em->finalized) throw std::invalid_argument("speq_em_scan_reads_device: bad or finalized histogram");
        scan_device_impl(em->dev, d_seq, d_qual, d_offsets, n_reads, p, d_counts, d_weights, em->d_mult, em->d_hi,
                         static_cast<hipStream_t>(stream));
    });
}

int speq_em_finalize(speq_em* em, uint32_t threads) {
    return speq::guarded([&] {
        if (!em) throw std::invalid_argument("speq_em_finalize: null argument");
        if (em->finalized) return;
        (void)threads;  // (the rows are built on the EM worker pool, em.cpp)
        DeviceGuard g(em->dev->device);
        HIP_OK(hipDeviceSynchronize());
        // only the positions that start a recorded interval come to the host, in position order (round 6: the two
        // whole per-position arrays were 80 MB at config 3, most of the CLI's 54 ms EM finalize)
        const uint64_t n = em->n;
        const uint32_t nb = (uint32_t)((n + EM_TILE - 1) / EM_TILE);
        hipStream_t st = em->dev->stream;
        uint32_t* d_cnt = nullptr;
        uint32_t* d_out = nullptr;
        HIP_OK(hipMalloc(&d_cnt, ((uint64_t)nb + 1) * 4));
        uint32_t nnz = 0;
        try {
            if (nb) {
                hipLaunchKernelGGL(k_em_count, dim3(nb), dim3(256), 0, st, em->d_mult, n, d_cnt);
                HIP_OK(hipGetLastError());
            }
            hipLaunchKernelGGL(k_em_scan, dim3(1), dim3(1024), 0, st, d_cnt, nb);
            HIP_OK(hipGetLastError());
            HIP_OK(hipMemcpyAsync(&nnz, d_cnt + nb, 4, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            // (lo, mult, hi) in one allocation, copied back by DMA into host memory page-locked for the copy (a
            // pageable copy of the three arrays took 8-9 ms at config 3)
            std::unique_ptr<uint32_t[]> tri(new uint32_t[3ull * std::max<uint32_t>(nnz, 1)]);
            if (nnz) {
                HIP_OK(hipMalloc(&d_out, (uint64_t)nnz * 12));
                hipLaunchKernelGGL(k_em_compact, dim3(nb), dim3(256), 0, st, em->d_mult, em->d_hi, n, d_cnt, d_out,
                                   d_out + nnz, d_out + 2ull * nnz);
                HIP_OK(hipGetLastError());
                // (the compaction first, then a synchronous copy: an asynchronous device-to-host copy on the
                // replica's stream paid about 8 ms of first-use cost in a `speq scan` process, this one 0.1 ms)
                HIP_OK(hipStreamSynchronize(st));
                const bool reg = hipHostRegister(tri.get(), (uint64_t)nnz * 12, hipHostRegisterDefault) == hipSuccess;
                if (!reg) (void)hipGetLastError();
                const hipError_t ce = hipMemcpy(tri.get(), d_out, (uint64_t)nnz * 12, hipMemcpyDeviceToHost);
                if (reg) (void)hipHostUnregister(tri.get());
                HIP_OK(ce);
            }
            (void)hipFree(d_cnt);
            if (d_out) (void)hipFree(d_out);
            d_cnt = d_out = nullptr;
            speq::em_build_rows(*em, tri.get(), tri.get() + nnz, tri.get() + 2ull * nnz, nnz);
        } catch (...) {
            (void)hipStreamSynchronize(st);
            if (d_cnt) (void)hipFree(d_cnt);
            if (d_out) (void)hipFree(d_out);
            throw;
        }
        (void)hipFree(em->d_mult);
        (void)hipFree(em->d_hi);
        em->d_mult = em->d_hi = nullptr;
    });
}

// Adds the histogram `src` recorded on another replica (same index; any GPU of this process, or the same one) into
// `dst`: src's arrays are copied to dst's device (peer copy over xGMI when the GPUs differ) and added by k_em_merge.
// src stays usable for nothing but speq_em_free afterwards.
int speq_em_merge(speq_em* dst, speq_em* src) {
    return speq::guarded([&] {
        if (!dst || !src || dst == src) throw std::invalid_argument("speq_em_merge: bad arguments");
        if (dst->finalized || src->finalized || !src->d_mult)
            throw std::invalid_argument("speq_em_merge: finalized or already merged histogram");
        if (dst->n != src->n || dst->G != src->G) throw std::invalid_argument("speq_em_merge: histograms of different indexes");
        {
            DeviceGuard gs(src->dev->device);
            HIP_OK(hipDeviceSynchronize());  // src's scans (any stream of its device) have completed
        }
        DeviceGuard g(dst->dev->device);
        HIP_OK(hipDeviceSynchronize());
        uint32_t *m = src->d_mult, *h = src->d_hi, *tmp = nullptr;
        if (src->dev->device != dst->dev->device) {
            HIP_OK(hipMalloc(&tmp, dst->n * 8));
            m = tmp;
            h = tmp + dst->n;
            HIP_OK(hipMemcpyPeerAsync(m, dst->dev->device, src->d_mult, src->dev->device, dst->n * 4, dst->dev->stream));
            HIP_OK(hipMemcpyPeerAsync(h, dst->dev->device, src->d_hi, src->dev->device, dst->n * 4, dst->dev->stream));
        }
        const uint64_t blocks = std::min<uint64_t>((dst->n + 1023) / 1024, 65536);
        hipLaunchKernelGGL(k_em_merge, dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(256), 0, dst->dev->stream,
                           dst->d_mult, dst->d_hi, m, h, dst->n);
        HIP_OK(hipGetLastError());
        HIP_OK(hipStreamSynchronize(dst->dev->stream));
        if (tmp) HIP_OK(hipFree(tmp));
        {
            DeviceGuard gs(src->dev->device);
            (void)hipFree(src->d_mult);
            (void)hipFree(src->d_hi);
        }
        src->d_mult = src->d_hi = nullptr;
    });
}

void speq_em_free(speq_em* em) {
    if (!em) return;
    if (em->d_mult) (void)hipFree(em->d_mult);
    if (em->d_hi) (void)hipFree(em->d_hi);
    delete em;
}

}  // extern "C"

namespace {
// Enqueues the .dat pass over shard `shard` of `n_shards` equal slices of the flattened reference windows (every
// text's fwd and rc windows in text order); the returned device buffer of window prefix sums must stay alive until
// the launch completes (freed by the caller after synchronizing `st`).
uint64_t* launch_ref_shard(speq_device_index* d, uint32_t k, uint32_t shard, uint32_t n_shards, uint64_t* d_u_ref,
                           uint64_t* d_tot_ref, hipStream_t st) {
    std::vector<uint64_t> cum(d->n_texts + 1, 0);
    for (uint32_t t = 0; t < d->n_texts; ++t) {
        const uint64_t L = d->text_start[t + 1] - d->text_start[t] - 1;  // minus separator
        cum[t + 1] = cum[t] + (L >= k ? L - k + 1 : 0);
    }
    const uint64_t all = cum[d->n_texts];
    const uint64_t w0 = all * shard / n_shards, w1 = all * (shard + 1) / n_shards;
    if (w1 == w0) return nullptr;
    uint64_t* d_cum = nullptr;
    HIP_OK(hipMalloc(&d_cum, cum.size() * 8));
    HIP_OK(hipMemcpyAsync(d_cum, cum.data(), cum.size() * 8, hipMemcpyHostToDevice, st));
    UnitSrc src{};
    src.seq = d->d_text;
    src.off = d->d_text_start;
    src.cum_win = d_cum;
    src.unit_group = d->d_text_group;
    src.n_units = d->n_texts;
    src.total_windows = w1 - w0;
    src.win_base = w0;
    src.end_adj = 1;
    src.k = k;
    src.buf_bytes = staging_bytes(k, std::max(d->ilp, d->ilp_kt ? d->ilp_kt : 2u));
    launch_scan(d, KM_REF, false, src, (w1 - w0 + 255) / 256, st, reinterpret_cast<unsigned long long*>(d_u_ref),
                reinterpret_cast<unsigned long long*>(d_tot_ref), nullptr);
    return d_cum;
}
}  // namespace

extern "C" {

int speq_ref_unique_device(speq_device_index* d, uint32_t k, uint64_t* d_u_ref, uint64_t* d_tot_ref, void* stream) {
    return speq::guarded([&] {
        if (!d || !d_u_ref || !d_tot_ref) throw std::invalid_argument("speq_ref_unique_device: null argument");
        if (k < 1 || k > MAX_K) throw std::invalid_argument("speq_ref_unique_device: k must be in [1, 4096]");
        DeviceGuard g(d->device);
        hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = the null (default) stream
        uint64_t* d_cum = launch_ref_shard(d, k, 0, 1, d_u_ref, d_tot_ref, st);
        if (!d_cum) return;
        HIP_OK(hipStreamSynchronize(st));  // d_cum is freed below
        HIP_OK(hipFree(d_cum));
    });
}

// Several replicas of one index (one per GPU of this process): replica i scans the i-th equal slice of the
// reference windows on its own stream, all concurrently; the per-group sums are added on the host (SURVEY 8(e):
// "the .dat pass shards reference records the same way" as the reads).
int speq_ref_unique_multi(speq_device_index* const* ds, uint32_t n_devices, uint32_t k, uint64_t* u_ref,
                          uint64_t* tot_ref) {
    return speq::guarded([&] {
        if (!ds || n_devices == 0 || !u_ref || !tot_ref) throw std::invalid_argument("speq_ref_unique_multi: null argument");
        if (k < 1 || k > MAX_K) throw std::invalid_argument("speq_ref_unique_multi: k must be in [1, 4096]");
        for (uint32_t i = 0; i < n_devices; ++i)
            if (!ds[i] || ds[i]->G != ds[0]->G || ds[i]->view.n != ds[0]->view.n)
                throw std::invalid_argument("speq_ref_unique_multi: replicas of different indexes");
        const uint32_t G = ds[0]->G;
        struct Shard {
            uint64_t* buf = nullptr;
            uint64_t* cum = nullptr;
            std::vector<uint64_t> host;
        };
        std::vector<Shard> sh(n_devices);
        auto release = [&] {
            for (uint32_t i = 0; i < n_devices; ++i) {
                DeviceGuard g(ds[i]->device);
                if (sh[i].buf || sh[i].cum) (void)hipStreamSynchronize(ds[i]->stream);
                if (sh[i].buf) (void)hipFree(sh[i].buf);
                if (sh[i].cum) (void)hipFree(sh[i].cum);
                sh[i].buf = sh[i].cum = nullptr;
            }
        };
        try {
            for (uint32_t i = 0; i < n_devices; ++i) {
                speq_device_index* d = ds[i];
                DeviceGuard g(d->device);
                HIP_OK(hipMalloc(&sh[i].buf, 2ull * G * 8));
                HIP_OK(hipMemsetAsync(sh[i].buf, 0, 2ull * G * 8, d->stream));
                sh[i].cum = launch_ref_shard(d, k, i, n_devices, sh[i].buf, sh[i].buf + G, d->stream);
                sh[i].host.assign(2ull * G, 0);
                HIP_OK(hipMemcpyAsync(sh[i].host.data(), sh[i].buf, 2ull * G * 8, hipMemcpyDeviceToHost, d->stream));
            }
            for (uint32_t i = 0; i < n_devices; ++i) {
                DeviceGuard g(ds[i]->device);
                HIP_OK(hipStreamSynchronize(ds[i]->stream));
            }
        } catch (...) {
            release();
            throw;
        }
        release();
        std::fill(u_ref, u_ref + G, 0);
        std::fill(tot_ref, tot_ref + G, 0);
        for (const Shard& s : sh)
            for (uint32_t g = 0; g < G; ++g) {
                u_ref[g] += s.host[g];
                tot_ref[g] += s.host[G + g];
            }
    });
}

int speq_ref_unique(speq_device_index* d, uint32_t k, uint64_t* u_ref, uint64_t* tot_ref) {
    return speq::guarded([&] {
        if (!d || !u_ref || !tot_ref) throw std::invalid_argument("speq_ref_unique: null argument");
        DeviceGuard g(d->device);
        const uint32_t G = d->G;
        uint64_t* buf = nullptr;
        HIP_OK(hipMalloc(&buf, 2ull * G * 8));
        HIP_OK(hipMemsetAsync(buf, 0, 2ull * G * 8, d->stream));
        int rc = speq_ref_unique_device(d, k, buf, buf + G, d->stream);
        if (rc != SPEQ_OK) {
            std::string msg = speq_last_error();
            (void)hipFree(buf);
            throw speq::DeviceError(msg);
        }
        HIP_OK(hipMemcpyAsync(u_ref, buf, G * 8, hipMemcpyDeviceToHost, d->stream));
        HIP_OK(hipMemcpyAsync(tot_ref, buf + G, G * 8, hipMemcpyDeviceToHost, d->stream));
        HIP_OK(hipStreamSynchronize(d->stream));
        HIP_OK(hipFree(buf));
    });
}

int speq_ref_unique_shard(speq_device_index* d, uint32_t k, uint32_t shard, uint32_t n_shards, uint64_t* u_ref,
                          uint64_t* tot_ref) {
    return speq::guarded([&] {
        if (!d || !u_ref || !tot_ref) throw std::invalid_argument("speq_ref_unique_shard: null argument");
        if (k < 1 || k > MAX_K) throw std::invalid_argument("speq_ref_unique_shard: k must be in [1, 4096]");
        if (n_shards == 0 || shard >= n_shards) throw std::invalid_argument("speq_ref_unique_shard: bad shard");
        DeviceGuard g(d->device);
        const uint32_t G = d->G;
        uint64_t* buf = nullptr;
        uint64_t* d_cum = nullptr;
        try {
            HIP_OK(hipMalloc(&buf, 2ull * G * 8));
            HIP_OK(hipMemsetAsync(buf, 0, 2ull * G * 8, d->stream));
            d_cum = launch_ref_shard(d, k, shard, n_shards, buf, buf + G, d->stream);
            HIP_OK(hipMemcpyAsync(u_ref, buf, G * 8, hipMemcpyDeviceToHost, d->stream));
            HIP_OK(hipMemcpyAsync(tot_ref, buf + G, G * 8, hipMemcpyDeviceToHost, d->stream));
            HIP_OK(hipStreamSynchronize(d->stream));
        } catch (...) {
            (void)hipStreamSynchronize(d->stream);
            if (d_cum) (void)hipFree(d_cum);
            if (buf) (void)hipFree(buf);
            throw;
        }
        if (d_cum) HIP_OK(hipFree(d_cum));
        HIP_OK(hipFree(buf));
    });
}

int speq_device_prepare(speq_device_index* d, uint32_t k, uint64_t* distinct_kmers, uint64_t* table_bytes,
                        double* build_ms) {
    return speq::guarded([&] {
        if (!d) throw std::invalid_argument("speq_device_prepare: null handle");
        if (k < 1 || k > MAX_K) throw std::invalid_argument("speq_device_prepare: k must be in [1, 4096]");
        if (const speq::AxTable* ax = speq::ensure_ax(d, k)) {  // the read scans' structures for k
            if (distinct_kmers) *distinct_kmers = ax->distinct;
            if (table_bytes) *table_bytes = ax->bytes;
            if (build_ms) *build_ms = ax->build_ms;
            return;
        }
        const speq_device_index::KmerTable* kt = ensure_ktab(d, k);
        if (distinct_kmers) *distinct_kmers = kt ? kt->distinct : 0;
        if (table_bytes) *table_bytes = kt ? kt->bytes : 0;
        if (build_ms) *build_ms = kt ? kt->build_ms : 0.0;
    });
}

int speq_device_set_tuning(speq_device_index* d, const char* key, int64_t value) {
    return speq::guarded([&] {
        if (!d || !key) throw std::invalid_argument("speq_device_set_tuning: null argument");
        const std::string k(key);
        if (k == "blocks_per_cu") {
            if (value < 0 || value > 8) throw std::invalid_argument("blocks_per_cu must be in [0, 8]");
            d->blocks_per_cu = (uint32_t)value;
        } else if (k == "ilp" || k == "ilp_local") {
            if (value != 1 && value != 2) throw std::invalid_argument(k + " must be 1 or 2");
            (k == "ilp" ? d->ilp : d->ilp_local) = (uint32_t)value;
        } else if (k == "grid_blocks") {
            if (value < 1 || value > (1 << 20)) throw std::invalid_argument("grid_blocks must be in [1, 2^20]");
            d->grid_blocks = (uint32_t)value;
        } else if (k == "fastq_gpu_parse") {
            if (value != 0 && value != 1) throw std::invalid_argument("fastq_gpu_parse must be 0 or 1");
            d->fastq_gpu = value != 0;
        } else if (k == "stream_lanes") {
            if (value < 1 || value > 8) throw std::invalid_argument("stream_lanes must be in [1, 8]");
            d->stream_lanes = (uint32_t)value;
        } else if (k == "sparse_prefix") {
            if (value < -1 || value > 1) throw std::invalid_argument("sparse_prefix must be -1 (auto), 0 or 1");
            if (value != 0) build_sparse(d);
            d->sparse_choice = (int)value;
        } else if (k == "grid_blocks_kt") {
            if (value < 1 || value > (1 << 20)) throw std::invalid_argument("grid_blocks_kt must be in [1, 2^20]");
            d->grid_blocks_kt = (uint32_t)value;
        } else if (k == "blocks_per_cu_kt") {
            if (value < 0 || value > 8) throw std::invalid_argument("blocks_per_cu_kt must be in [0, 8]");
            d->blocks_per_cu_kt = (uint32_t)value;
        } else if (k == "kt_pipeline") {
            if (value != 0 && value != 1) throw std::invalid_argument("kt_pipeline must be 0 or 1");
            d->kt_pipeline = value != 0;
        } else if (k == "ilp_kt") {
            if (value != 0 && value != 1 && value != 2 && value != 4)
                throw std::invalid_argument("ilp_kt must be 0 (auto), 1, 2 or 4");
            d->ilp_kt = (uint32_t)value;
        } else if (k == "kt_compact") {
            if (value != 0 && value != 1) throw std::invalid_argument("kt_compact must be 0 or 1");
            d->kt_compact = value != 0;
        } else if (k == "kt_load8") {
            if (value < 10 || value > 90) throw std::invalid_argument("kt_load8 must be in [10, 90] (percent)");
            d->kt_load8 = (uint32_t)value;
        } else if (k == "kt_slots") {
            if (value < 2 || value > 16) throw std::invalid_argument("kt_slots must be in [2, 16]");
            d->kt_slots = (uint32_t)value;
        } else if (k == "ax_scan") {
            if (value != 0 && value != 1) throw std::invalid_argument("ax_scan must be 0 or 1");
            d->ax_scan = value != 0;
        } else if (k == "ax_mproof") {
            if (value < 0 || value > 2) throw std::invalid_argument("ax_mproof must be 0, 1 or 2");
            d->ax_mproof = (uint32_t)value;
        } else if (k == "ax_load") {
            if (value < 10 || value > 90) throw std::invalid_argument("ax_load must be in [10, 90] (percent)");
            std::lock_guard<std::mutex> lk(d->ax_mu);
            if (!d->axtabs.empty() && (uint32_t)value != speq::ax_effective_load(d))
                throw std::invalid_argument("ax_load must be set before the first scan");
            d->ax_load = (uint32_t)value;
        } else if (k == "grid_blocks_ax") {
            if (value < 1 || value > 65535) throw std::invalid_argument("grid_blocks_ax must be in [1, 65535]");
            d->grid_blocks_ax = (uint32_t)value;
        } else if (k == "blocks_per_cu_ax") {
            if (value < 0 || value > 8) throw std::invalid_argument("blocks_per_cu_ax must be in [0, 8]");
            d->blocks_per_cu_ax = (uint32_t)value;
        } else if (k == "ax_generations") {
            if (value < 1 || value > 16) throw std::invalid_argument("ax_generations must be in [1, 16]");
            d->ax_generations = (uint32_t)value;
        } else if (k == "kmer_table") {
            if (value != 0 && value != 1) throw std::invalid_argument("kmer_table must be 0 or 1");
            d->kmer_table = value != 0;
        } else if (k == "prefix_level") {
            if (value < -1 || value > 2) throw std::invalid_argument("prefix_level must be -1 (auto) or 0..2");
            if (value >= 0 && (d->prefix_level[value] == nullptr && value > 0))
                throw std::invalid_argument("prefix_level: the index has no table at that level");
            d->prefix_choice = (int)value;
            d->view.prefix = value > 0 ? d->prefix_level[value] : d->prefix_level[0];
            d->view.q = d->prefix_level[0] ? d->base_q - (uint32_t)(value > 0 ? value : 0) : 0;
        } else {
            throw std::invalid_argument("speq_device_set_tuning: unknown key " + k);
        }
    });
}

int speq_device_get_tuning(const speq_device_index* d, const char* key, int64_t* value) {
    return speq::guarded([&] {
        if (!d || !key || !value) throw std::invalid_argument("speq_device_get_tuning: null argument");
        const std::string k(key);
        if (k == "blocks_per_cu") *value = d->blocks_per_cu;
        else if (k == "ilp") *value = d->ilp;
        else if (k == "ilp_local") *value = d->ilp_local;
        else if (k == "grid_blocks") *value = d->grid_blocks;
        else if (k == "prefix_level") *value = d->prefix_choice;
        else if (k == "sparse_prefix") *value = d->sparse_choice;
        else if (k == "fastq_gpu_parse") *value = d->fastq_gpu ? 1 : 0;
        else if (k == "stream_lanes") *value = d->stream_lanes;
        else if (k == "kmer_table") *value = d->kmer_table ? 1 : 0;
        else if (k == "ilp_kt") *value = d->ilp_kt;
        else if (k == "kt_pipeline") *value = d->kt_pipeline ? 1 : 0;
        else if (k == "blocks_per_cu_kt") *value = d->blocks_per_cu_kt;
        else if (k == "grid_blocks_kt") *value = d->grid_blocks_kt;
        else if (k == "kt_slots") *value = d->kt_slots;
        else if (k == "kt_compact") *value = d->kt_compact ? 1 : 0;
        else if (k == "kt_load8") *value = d->kt_load8;
        else if (k == "ax_scan") *value = d->ax_scan ? 1 : 0;
        else if (k == "last_kernel") *value = d->last_kernel;
        else if (k == "ax_mproof") *value = d->ax_mproof;
        else if (k == "ax_load") *value = speq::ax_effective_load(d);
        else if (k == "grid_blocks_ax") *value = d->grid_blocks_ax;
        else if (k == "blocks_per_cu_ax") *value = d->blocks_per_cu_ax;
        else if (k == "ax_generations") *value = d->ax_generations;
        else throw std::invalid_argument("speq_device_get_tuning: unknown key " + k);
    });
}

int speq_timing_enable(speq_device_index* d, int on) {
    return speq::guarded([&] {
        if (!d) throw std::invalid_argument("speq_timing_enable: null handle");
        d->timing = on != 0;
    });
}

int speq_timing_read(speq_device_index* d, double* total_ms, uint64_t* launches) {
    return speq::guarded([&] {
        if (!d || !total_ms || !launches) throw std::invalid_argument("speq_timing_read: null argument");
        DeviceGuard g(d->device);
        double ms = 0.0;
        std::lock_guard<std::mutex> lk(d->events_mu);
        for (auto& e : d->events) {
            HIP_OK(hipEventSynchronize(e.second));
            float t = 0.f;
            HIP_OK(hipEventElapsedTime(&t, e.first, e.second));
            ms += t;
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        *total_ms = ms;
        *launches = d->events.size();
        d->events.clear();
    });
}

}  // extern "C"

namespace speq {
void em_clear(speq_em* em) {
    if (!em) return;
    if (em->finalized) throw std::logic_error("speq: EM histogram already finalized");
    DeviceGuard g(em->dev->device);
    HIP_OK(hipMemset(em->d_mult, 0, em->n * 4));
    HIP_OK(hipMemset(em->d_hi, 0, em->n * 4));
}
}  // namespace speq


// ---- internal entry points for the streaming pipeline (pipeline.cpp; scan_internal.hpp) ----
namespace speq {
void launch_reads_scan(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual, const uint64_t* d_offsets,
                       uint64_t n_reads, const speq_scan_params* p, uint64_t* d_counts, double* d_weights,
                       uint32_t* em_mult, uint32_t* em_hi, void* stream) {
    scan_device_impl(d, d_seq, d_qual, d_offsets, n_reads, p, d_counts, d_weights, em_mult, em_hi,
                     static_cast<hipStream_t>(stream));
}
int device_ordinal(const speq_device_index* d) { return d->device; }
bool device_fastq_gpu(const speq_device_index* d) { return d->fastq_gpu; }
uint32_t device_stream_lanes(const speq_device_index* d) { return d->stream_lanes; }
uint32_t device_groups(const speq_device_index* d) { return d->G; }
uint64_t device_text_len(const speq_device_index* d) { return d->view.n; }
}  // namespace speq

namespace speq {
// Loads this translation unit's code object onto the current device (HIP loads a code object at the first use of
// one of its kernels: 30-55 ms for the scan kernels' on the first launch of a `speq scan` run; speq_device_warmup).
void warm_module_scan_kernels() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_ktab_keys));
}
}  // namespace speq
