// Anchor-and-extend read scan (k_scan_ax) and its per-k structures, for gfx950 (MI355X). DESIGN.md §4e.
//
// Replaces, for every read window, the reference's `search(f_kmers, fm_index, cfg)` + the first-hit tally
// (/root/reference/src/fm_scanner.cpp:153-196 global, :426-471 local, :665-729 paired, :916-962 paired local).
//
// Why: consecutive windows of a read that matches the reference are consecutive positions of the reference text, and
// whether a k-mer is unique to one group is a property of the k-mer, i.e. of ANY of its occurrences. A k-mer that
// occurs at text position p occurs in the group of p's text, so its class is one of four 2-bit codes relative to that
// text: OWN (every occurrence is in the group of p's text), MULTI (occurrences in >= 2 groups), SENT (the window holds
// an N inside one text) or END (the window crosses a text end). Per k the replica keeps
//   * `gran`: per 32 text positions one 16-B granule {2-bit text of the 32 positions, class plane 0, class plane 1}
//     — a run over the rest of a read is up to six consecutive 16-B loads of ONE array (text and classes together);
//   * `atab`: a hash table of one representative position per distinct k-mer, each slot {position, 16-bit
//     fingerprint, group of the position's text};
//   * a blocked Bloom filter of the distinct k-mers.
// A lane takes one READ: it looks one window up (the anchor: bucket -> fingerprint -> representative p and its
// text's group), then compares the read with the text at p, 64 windows at a time (one XOR per 32 bases), and tallies
// the matched OWN windows to the run's group. A mismatch (a SNP against the representative, or a sequencing error)
// ends the run and the next window is looked up again; so does an END window (the run would leave p's text).
// Every verdict is exact: a window is classified from its class at p' only after its k bases were compared equal
// with text[p', p' + k) (SENT windows, whose text holds an N coded as A, are never classified from the text: they are
// looked up), and a window is absent only after its key's chain in the anchor table ran into an empty slot without a
// verified match (or its bits are missing from the Bloom filter, which holds every k-mer of the texts).
//
// Windows whose anchor lookup finds nothing (the k windows over a sequencing error) and SENT windows are DEFERRED:
// the wave collects them in LDS and, after the per-read pass, tests them against the Bloom filter (four per lane per
// round trip) and looks the survivors up one per lane, so one erroneous read does not hold its wave for k lookups.
//
// What bounds it (profiles/r02, r03): the per-CU vector-memory path, which serves the lanes' scattered loads one cache
// line per lane and instruction. So a run's text and classes come from one array (at most six 16-B loads that cover
// the rest of the read, where r02 loaded four 8-B text words and five class dwords per 64 windows), a clean read is
// one lookup and one run, a load group is issued only when some lane of the wave needs it, and one iteration costs
// one round trip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "device_index.hpp"
#include "fm_index.hpp"
#include "scan_device.hpp"
#include "scan_internal.hpp"
#include "speq_scan.h"
#include "ax_common.hpp"

namespace {

using namespace speq_dev;

// ---------------------------------------------------------------------------------------------------------------
// Per-k structures
// ---------------------------------------------------------------------------------------------------------------

// 2-bit text (A C G T = 0..3; separators, terminator and N as 0) and the bitmap of non-ACGT positions, for the
// whole FM text; positions >= n are "bad". One thread per 64 positions.
__global__ void k_ax_text2(const uint8_t* __restrict__ text, uint64_t n, uint64_t* __restrict__ t2,
                           uint64_t* __restrict__ tbad, uint64_t n_words64) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words64;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = 0, bad = 0;
        for (uint32_t i = 0; i < 64; ++i) {
            const uint64_t pos = w * 64 + i;
            const uint32_t c = pos < n ? text[pos] : 0u;
            const bool acgt = c >= 2u && c <= 5u;
            const uint64_t code = acgt ? (uint64_t)(c - 2u) : 0ull;
            if (i < 32) lo |= code << (2 * i);
            else hi |= code << (2 * (i - 32));
            bad |= (uint64_t)(acgt ? 0u : 1u) << i;
        }
        t2[2 * w] = lo;
        t2[2 * w + 1] = hi;
        tbad[w] = bad;
    }
}

// Backward search of the k symbols text[pos .. pos + k) (all ACGT): q-mer table, then three/two/one-symbol LF steps
// (search_lds with the symbols read from the text), then the label-run classification.
__device__ int ax_search_text(const DevView& I, const Rsrc& R, const uint8_t* __restrict__ t, uint32_t k,
                              uint32_t& lo_out, uint32_t& hi_out) {
    uint32_t lo = 0, hi = I.n;
    int32_t s = (int32_t)k;
    auto sym = [&](int32_t i) -> uint32_t { return (uint32_t)t[i] - 2u; };
    if (I.q != 0u && k >= I.q) {
        uint32_t code = 0;
        for (uint32_t i = k - I.q; i < k; ++i) code = (code << 2) | sym((int32_t)i);
        const uint2 e = prefix_lookup(I, code);
        lo = e.x;
        hi = e.y;
        s -= (int32_t)I.q;
    }
    if (I.occ3 != nullptr) {
        const int32_t rem = s % 3;
        if (rem == 1 && lo < hi) {
            lf_step(I, R.occ, sym(s - 1), lo, hi);
            --s;
        } else if (rem == 2 && lo < hi) {
            lf_step(I, R.occ2, sym(s - 2) * 4u + sym(s - 1), lo, hi);
            s -= 2;
        }
        while (s > 0 && lo < hi) {
            lf_step(I, R.occ3, sym(s - 3) * 16u + sym(s - 2) * 4u + sym(s - 1), lo, hi);
            s -= 3;
        }
    } else if (I.occ2 != nullptr) {
        if ((s & 1) && lo < hi) {
            lf_step(I, R.occ, sym(s - 1), lo, hi);
            --s;
        }
        while (s > 0 && lo < hi) {
            lf_step(I, R.occ2, sym(s - 2) * 4u + sym(s - 1), lo, hi);
            s -= 2;
        }
    } else {
        while (s > 0 && lo < hi) {
            lf_step(I, R.occ, sym(s - 1), lo, hi);
            --s;
        }
    }
    lo_out = lo;
    hi_out = hi;
    return lo < hi ? classify(I, R, lo, hi) : -1;
}

// Pass A: the class code of the k-mer at every text position (one byte per position, packed into granules by pass
// B), and one representative position per distinct k-mer (the first to claim owner[lo] of its SA interval).
//
// The representative is the occurrence at the MEDIAN rank of the k-mer's SA interval, SA[(lo + hi -
// 1) / 2]. Within the interval the suffixes are sorted by the text that follows the k-mer, so occurrences that share
// their continuation form contiguous groups, and whenever one continuation is shared by more than half of the
// occurrences, the median lies in it, base after base: the representative follows the consensus of the records that
// contain the k-mer. A read run from it breaks only where the read's record leaves that consensus (its own SNPs),
// not wherever an arbitrary representative's record has one — fewer lookups and runs per read (simulated on config 2:
// 1.99 -> 1.76 runs per read against a uniformly random occurrence, 3.13 for the lowest position; the first
// claimant of round 3 leaned towards the lowest: config 5 measured 3.6). sa == nullptr (the replica's suffix array did
// not fit the free HBM): the first thread to claim the interval.
__global__ void k_ax_classify(DevView I, const uint8_t* __restrict__ text, const uint64_t* __restrict__ tbad,
                              uint64_t n, uint32_t k, uint8_t* __restrict__ codes, uint32_t* __restrict__ owner,
                              const uint32_t* __restrict__ sa, unsigned long long* __restrict__ n_distinct) {
    const Rsrc R = make_rsrc(I);
    unsigned long long claimed = 0;
    for (uint64_t pos = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; pos < n;
         pos += (uint64_t)gridDim.x * blockDim.x) {
        // valid window: no non-ACGT symbol in [pos, pos + k) (positions >= n are bad)
        bool valid = true;
        for (uint64_t b = pos; b < pos + k && valid;) {
            const uint64_t w = b >> 6, sh = b & 63u;
            const uint64_t span = (64u - sh < pos + k - b) ? 64u - sh : pos + k - b;
            const uint64_t m = span == 64u ? ~0ull : ((1ull << span) - 1ull);
            valid = ((tbad[w] >> sh) & m) == 0;
            b += span;
        }
        if (!valid) {  // END when the window reaches a separator / the terminator / past n, else SENT (an N)
            bool end = pos + k > n;
            for (uint32_t i = 0; i < k && !end; ++i) end = text[pos + i] <= 1u;
            codes[pos] = (uint8_t)(end ? AX_END : AX_SENT);
            continue;
        }
        uint32_t lo = 0, hi = 0;
        const int g = ax_search_text(I, R, text + pos, k, lo, hi);
        // g == -1 cannot happen: the window occurs at pos; g >= 0 is the group of pos's text
        codes[pos] = (uint8_t)(g >= 0 ? AX_OWN : AX_MULTI);
        const uint32_t rp = sa != nullptr ? sa[lo + (hi - lo - 1u) / 2u] : (uint32_t)pos;
        if (atomicCAS(&owner[lo], AX_EMPTY, rp) == AX_EMPTY) ++claimed;
    }
    if (claimed) atomicAdd(n_distinct, claimed);
}

// EM scans only (built on the first EM scan of k): every text position whose k-mer is MULTI (granule class planes)
// records its SA interval, mlo[pos] = its start and mhi[start] = its end, for the EM histogram of the scan.
__global__ void k_ax_em_intervals(DevView I, const uint8_t* __restrict__ text, const u32x4* __restrict__ gran,
                                  uint64_t n, uint32_t k, uint32_t* __restrict__ mlo, uint32_t* __restrict__ mhi) {
    const Rsrc R = make_rsrc(I);
    for (uint64_t pos = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; pos < n;
         pos += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 gv = gran[pos >> 5];
        const uint32_t b = (uint32_t)pos & 31u;
        if ((((gv[2] >> b) & 1u) | (((gv[3] >> b) & 1u) << 1)) != AX_MULTI) continue;
        uint32_t lo = 0, hi = 0;
        ax_search_text(I, R, text + pos, k, lo, hi);  // a MULTI window is all ACGT and occurs at pos
        mlo[pos] = lo;
        mhi[lo] = hi;
    }
}

// Pass B: granule b = {t2 word b (positions 32b .. 32b + 31), class plane 0, class plane 1}; positions >= n are END.
__global__ void k_ax_pack(const uint64_t* __restrict__ t2, uint64_t t2_words, const uint8_t* __restrict__ codes,
                          uint64_t n, u32x4* __restrict__ gran, uint64_t n_gran) {
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n_gran;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = b < t2_words ? t2[b] : 0ull;
        uint32_t p0 = 0, p1 = 0;
        for (uint32_t i = 0; i < 32; ++i) {
            const uint64_t pos = 32 * b + i;
            const uint32_t c = pos < n ? codes[pos] : AX_END;
            p0 |= (c & 1u) << i;
            p1 |= (c >> 1) << i;
        }
        u32x4 v;
        v[0] = (uint32_t)t;
        v[1] = (uint32_t)(t >> 32);
        v[2] = p0;
        v[3] = p1;
        gran[b] = v;
    }
}

// aligned little-endian 2-bit words of the text starting at base p
template <int NW>
__device__ __forceinline__ void ax_text_words(const uint64_t* __restrict__ t2, uint64_t p, uint64_t (&w)[NW]) {
    const uint64_t w0 = p >> 5;
    const uint32_t sh = 2u * (uint32_t)(p & 31u);
    uint64_t raw[NW + 1];
#pragma unroll
    for (int i = 0; i <= NW; ++i) raw[i] = t2[w0 + i];
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = funnel(raw[i], raw[i + 1], sh);
}

// Pass C: every representative position inserts {position | (fingerprint << 16 | group of its text) << 32} into the
// anchor table (8 slots per 64-B bucket, first empty slot in order, linear probing over buckets; no deletions) and
// sets its filter bits.
__global__ void k_ax_insert(const uint32_t* __restrict__ owner, uint64_t n, const uint64_t* __restrict__ t2, uint32_t k,
                            const uint64_t* __restrict__ text_start, const int32_t* __restrict__ text_group,
                            uint32_t n_texts, unsigned long long* __restrict__ atab, uint64_t nb,
                            unsigned long long* __restrict__ filt, uint64_t nf) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = owner[i];
        if (p == AX_EMPTY) continue;
        uint64_t w[4];
        ax_text_words<4>(t2, p, w);
        const uint64_t h = ax_hash<4>(w, k);
        atomicOr(&filt[ax_fword(h, nf)], (unsigned long long)ax_fbits(h));
        uint32_t lo = 0, hi = n_texts;  // the last text t with text_start[t] <= p
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) / 2u;
            if (text_start[mid] <= p) lo = mid;
            else hi = mid;
        }
        const uint32_t grp = (uint32_t)text_group[lo] & 0xFFFFu;
        const unsigned long long v = ((unsigned long long)((ax_fp(h) << 16) | grp) << 32) | p;
        uint32_t b = ax_bucket(h, nb);
        for (bool placed = false; !placed; b = (b + 1u == nb) ? 0u : b + 1u)
            for (uint32_t j = 0; j < 8u && !placed; ++j)
                placed = atomicCAS(&atab[(uint64_t)b * 8u + j], AX_SLOT_EMPTY, v) == AX_SLOT_EMPTY;
    }
}

// Pass D: the m-mer filter — a blocked Bloom filter of every m-mer of the texts that holds no non-ACGT symbol (both
// strands: the texts are [fwd_r, rc_r]). A window that contains an m-mer whose bits are missing cannot occur in the
// texts (every occurrence of the window would contain an occurrence of the m-mer), so the scan proves the windows
// around a mismatch absent with a few m-mer probes instead of deferring each (k_scan_ax, lane state 4).
__global__ void k_ax_mfilter(const uint64_t* __restrict__ t2, const uint64_t* __restrict__ tbad, uint64_t n,
                             uint32_t m, unsigned long long* __restrict__ mf, uint64_t nmf) {
    for (uint64_t pos = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; pos + m <= n;
         pos += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = pos >> 6, sh = pos & 63u;
        const uint64_t bad = sh + m <= 64u ? (tbad[w] >> sh) : ((tbad[w] >> sh) | (tbad[w + 1] << (64u - sh)));
        if ((bad & ((m == 64u) ? ~0ull : ((1ull << m) - 1ull))) != 0) continue;
        uint64_t x[1];
        ax_text_words<1>(t2, pos, x);
        const uint64_t h = ax_hash<1>(x, m);
        atomicOr(&mf[ax_fword(h, nmf)], (unsigned long long)ax_fbits(h));
    }
}

// m of the m-mer filter of a text of n symbols for k-mers: the smallest m >= 12 with 4^m >= 200 n (a random m-mer
// then occurs in the text with probability <= 1 %, so an m-mer over a sequencing error is almost always absent),
// and only when one probe covers at least AX_MP_COVER windows (k - m + 1): a probe iteration delays its lane by one
// round trip, which the deferred windows it saves repay from about 12 on (config 2, k = 21, m = 14: 8 windows per
// probe, 1-3 % slower with the proofs; k = 31, m = 16-18 and k = 70 win: profiles/r05/ab_mproof*.jsonl); 0 = none
constexpr uint32_t AX_MP_COVER = 12;
static uint32_t ax_mproof_m(uint64_t n, uint32_t k) {
    uint32_t m = 12;
    while (m < 32u && (double)(1ull << (2u * m)) < 200.0 * (double)n) ++m;
    return k + 1u >= m + AX_MP_COVER ? m : 0u;
}

// ---------------------------------------------------------------------------------------------------------------
// The scan
// ---------------------------------------------------------------------------------------------------------------

// HW = 2-bit words of one k-mer (its hash): 1 (k <= 32), 2 (k <= 64), 3 (k <= 96), 4 (k <= 128); a phase-2 verification loads the
// HW + 1 granules that cover k bases at any offset in the first.
//
// Persistent lanes: a wave takes the units (reads, or mate pairs) of its groups of 64 in order; every lane works on
// one unit at a time, piece by piece (a read segment of at most AX_CAP bases; a pair's mates one after the other),
// and takes the next unit from the wave's pool when it is done. A lane's chain of dependent round trips depends on
// its read (one lookup and one run for a clean read; one more of each per mismatch against the representative's text
// or per sequencing error), so lanes that finish early are refilled in batches (SPEQ_AX_REFILL lanes at a time:
// coalesced staging of their next pieces) instead of idling until the wave's slowest read is done. Deferred windows
// (phase 2) are resolved by the whole wave when SPEQ_AX_BLOCKED finished lanes wait for theirs (their slots hold the
// bases the deferred entries refer to) or when the list fills up.
template <int MODE, bool PAIRED, bool LDS_HIST, bool EM, int HW, bool STATS>
__global__ __launch_bounds__(AX_THREADS, (ax_min_waves<MODE, HW, EM, STATS>())) void k_scan_ax(AxView A, UnitSrc src,
                                                                                  unsigned long long* __restrict__ out_a,
                                                                                  double* __restrict__ out_w) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = A.G, k = src.k;
    const uint32_t hist_words = LDS_HIST ? ((MODE == KM_GLOBAL) ? G : 2u * G) : 0u;
    const uint32_t hist_bytes = (hist_words * 8u + 15u) & ~15u;
    unsigned long long* hA = reinterpret_cast<unsigned long long*>(smem);
    double* hW = reinterpret_cast<double*>(hA + G);
    // KM_LOCAL: ftab[min(byte, 75)] = fl(1 / lut[q]) of the quality byte's rank q (bytes <= 33 rank 0, >= 74 rank 41;
    // entry 76 = 1.0, the factor of a byte outside a product), wtab[q] = the weight of a window of k bytes of rank q
    double* ftab = reinterpret_cast<double*>(smem + hist_bytes);
    double* wtab = ftab + AX_FTAB;
    const uint32_t qtab_bytes = MODE == KM_LOCAL ? QTAB_BYTES : 0u;
    constexpr uint32_t WAVE_BYTES = ax_wave_bytes<MODE>();
    unsigned char* wb = smem + hist_bytes + qtab_bytes + wid * WAVE_BYTES;
    uint32_t* codes = reinterpret_cast<uint32_t*>(wb);                       // [AX_CHUNKS][64]
    uint64_t* vw = reinterpret_cast<uint64_t*>(codes + AX_CHUNKS * 64u);     // [AX_VWW][64]
    uint16_t* bad16 = reinterpret_cast<uint16_t*>(vw);                       // staging: see bad_at
    uint16_t* chg = reinterpret_cast<uint16_t*>(vw + AX_VWW * 64u);          // [AX_CHUNKS][64] (local)
    uint8_t* off0s = reinterpret_cast<uint8_t*>(chg + (MODE == KM_LOCAL ? AX_CHUNKS * 64u : 0u));   // [64]
    uint16_t* defl = reinterpret_cast<uint16_t*>(off0s + 64);                // [AX_DEF]
    constexpr uint32_t AX_DEF = ax_def<MODE>();
    uint32_t* defn = reinterpret_cast<uint32_t*>(defl + AX_DEF);             // [2]: entries, survivors
    // the wave's sums of passing windows (T) and ambiguous units, u64 (8-B aligned: every array before is a multiple
    // of 8 B), added to by the lanes' LDS atomics as they go (no per-lane registers held for them)
    unsigned long long* wsum = reinterpret_cast<unsigned long long*>(defn + 2);  // [2]
    int32_t* ambf = reinterpret_cast<int32_t*>(defn + 6);                    // [64] first counted group
    int32_t* ambd = ambf + 64;                                               // [64] another group seen
    uint32_t* wl = reinterpret_cast<uint32_t*>(ambd + 64);                   // [AX_WL] (local)
    uint32_t* wlm = wl + AX_WL;                                              // [64] (local)
    uint8_t* ownb = reinterpret_cast<uint8_t*>(MODE == KM_LOCAL ? wlm + 64 : wl);  // [ax_ownb] staging owner map

    if (MODE == KM_LOCAL)
        for (uint32_t i = threadIdx.x; i < AX_FTAB; i += AX_THREADS) {
            const int q = (int)i - 33;
            ftab[i] = i == AX_FONE ? 1.0 : src.qlut[2 * (q < 0 ? 0 : (q > 41 ? 41 : q)) + 1];
            if (i < QLUT_LEN) {
                const double lut = src.qlut[2 * i], inv = src.qlut[2 * i + 1];
                double x = 1.0;  // fm_scanner.cpp:454, k bases of quality i
                for (uint32_t j = 0; j < k; ++j) x = div_rn(x, lut, inv);
                wtab[i] = x;
            }
        }
    if (LDS_HIST)
        for (uint32_t i = threadIdx.x; i < hist_words; i += AX_THREADS) hA[i] = 0ull;
    if (lane == 0) {
        defn[0] = defn[1] = 0u;
        wsum[0] = wsum[1] = 0ull;
    }
    __syncthreads();
    unsigned long long* gU = out_a + 2;

    // every table is read through a buffer descriptor: 16-B loads need only dword alignment, and a lane that has
    // nothing to load gets an out-of-range offset, which issues no memory request
    const __amdgpu_buffer_rsrc_t rs_gran =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.gran, (short)0, (int)(uint32_t)A.gran_bytes, 0x00020000);
    // (the anchor table's descriptor also covers the m-mer filter after it: 16-B loads of its 8-B words)
    const __amdgpu_buffer_rsrc_t rs_atab = __builtin_amdgcn_make_buffer_rsrc(
        (void*)A.atab, (short)0, (int)(uint32_t)(A.nb * 64u + (A.m != 0u ? A.nmf * 8u + 16u : 0u)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_filt =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.filt, (short)0, (int)(uint32_t)(A.nf * 8u), 0x00020000);
    const uint64_t NWV = (uint64_t)gridDim.x * AX_WPB;
    const uint64_t gw = (uint64_t)blockIdx.x * AX_WPB + wid;
    const uint64_t nu = PAIRED ? src.n_units / 2 : src.n_units;  // units: reads, or mate pairs
    const uint32_t segw = AX_CAP - k + 1u;  // windows per segment
    const uint32_t qt = 33u + src.cutoff;   // Phred+33 byte <= qt  <=>  clamp(q, 0, 41) <= cutoff (cutoff < 41)
    const uint32_t qt4 = (qt > 0x7Fu ? 0x7Fu : qt) * 0x01010101u;
    const uint32_t allbad = src.cutoff >= 41u ? 0x80808080u : 0u;  // every window fails the quality filter

    // diagnostic counters (STATS only; wave-level ones are counted by lane 0)
    uint32_t s_iter = 0, s_lk = 0, s_rn = 0, s_lkw = 0, s_rnw = 0, s_rwin = 0, s_def = 0, s_fp = 0, s_p2 = 0,
             s_p2v = 0, s_ch = 0, s_seg = 0, s_qb = 0, s_tal = 0, s_rg = 0, s_spl = 0, s_b4 = 0, s_b16 = 0, s_b32 = 0,
             s_b64 = 0, s_p2n = 0, s_p2r = 0;
    // section clocks (STATS only; wave-uniform, kept by every lane, reported by lane 0)
    uint64_t c_ref = 0, c_lk = 0, c_rn = 0, c_p2 = 0, c_p2f = 0, c_rpre = 0, c_rstg = 0, c_t0 = STATS ? clock64() : 0ull, c_s = 0;

    auto add_count = [&](uint32_t g, uint32_t cnt, double wsum) {
        if (LDS_HIST) {
            atomicAdd(&hA[g], (unsigned long long)cnt);
            if (MODE == KM_LOCAL && wsum != 0.0) atomicAdd(&hW[g], wsum);
        } else {
            atomicAdd(&gU[g], (unsigned long long)cnt);
            if (MODE == KM_LOCAL && wsum != 0.0) atomicAdd(&out_w[g], wsum);
        }
    };
    auto add_weight = [&](uint32_t g, double w) {
        if (LDS_HIST) atomicAdd(&hW[g], w);
        else atomicAdd(&out_w[g], w);
    };
    // 32 bases (64 bits) of slot o from slot position pos
    auto slot64 = [&](uint32_t o, uint32_t pos) -> uint64_t {
        const uint32_t d = pos >> 4, sh = 2u * (pos & 15u);
        const uint32_t w0 = d < AX_CHUNKS ? codes[d * 64u + o] : 0u;
        const uint32_t w1 = d + 1u < AX_CHUNKS ? codes[(d + 1u) * 64u + o] : 0u;
        const uint32_t w2 = d + 2u < AX_CHUNKS ? codes[(d + 2u) * 64u + o] : 0u;
        return u64of(alignbit(w1, w0, sh), alignbit(w2, w1, sh));
    };
    auto read_words = [&](uint32_t o, uint32_t pos, uint64_t(&w)[HW]) {  // HW code words of slot o at pos
        if (HW <= 2) {  // (HW = 2: the shared reads below hold more registers at once and spill)
#pragma unroll
            for (int i = 0; i < HW; ++i) w[i] = slot64(o, pos + 32u * (uint32_t)i);
            return;
        }
        // the 2 HW + 1 slot words that cover them, each read once (consecutive 64-bit words share a slot word)
        const uint32_t d = pos >> 4, sh = 2u * (pos & 15u);
        uint32_t c[2 * HW + 1];
#pragma unroll
        for (int i = 0; i <= 2 * HW; ++i) c[i] = d + (uint32_t)i < AX_CHUNKS ? codes[(d + (uint32_t)i) * 64u + o] : 0u;
#pragma unroll
        for (int i = 0; i < HW; ++i) w[i] = u64of(alignbit(c[2 * i + 1], c[2 * i], sh), alignbit(c[2 * i + 2], c[2 * i + 1], sh));
    };
    auto vbits = [&](uint32_t o, uint32_t b) -> uint64_t {  // read o's valid-window bits b .. b + 63 (0 past the end)
        const uint32_t w0 = b >> 6, s6 = b & 63u;
        const uint64_t lo = w0 < AX_VWW ? vw[w0 * 64u + o] : 0ull;
        const uint64_t hi = w0 + 1u < AX_VWW ? vw[(w0 + 1u) * 64u + o] : 0ull;
        return funnel(lo, hi, s6);
    };
    auto next_valid = [&](uint32_t o, uint32_t j, uint32_t end) -> uint32_t {  // first valid window of read o in
        for (uint32_t b = j; b < end; b += 64u) {                             // [j, end), else end
            const uint64_t v = vbits(o, b);
            if (v) return min(b + (uint32_t)__builtin_ctzll(v), end);
        }
        return end;
    };
    // the factor of quality byte x (its low 8 bits): fl(1 / lut[q]) for its rank q (phred42: bytes below '!' rank 0,
    // above 'J' rank 41)
    auto fac = [&](uint32_t x) -> double { return ftab[min(x & 0xFFu, AX_FONE - 1u)]; };
    // the summed weights of the windows t (bits of mask, t < 8) of a block whose first window's first quality byte is
    // src.qual[qo] (k >= 8). fm_scanner.cpp:454 divides 1 by the lut values of a window's k qualities in turn; here
    // window t (bytes t .. t + k - 1 of the block) is S[t] P[t], S[t] the product of the reciprocals ftab of bytes
    // t .. 7 (a chain from byte 7 down), P[t] that of bytes 8 .. k + t - 1 (the middle product M of bytes 8 .. k - 1,
    // then one byte more per window): a product tree over the window's k factors, k - 1 roundings, within 3 k 2^-53 of
    // the reference's quotient (relative), and added to the block's sum by one fma (exact product).
    // Every quality dword of the block is loaded before the first product (one round trip; the middle product's next
    // 16 bytes are loaded while the current 16 are multiplied, k > 24), and the factors' LDS reads issue in groups
    // rather than one wait per factor. Dwords past the last byte of the last window in the mask are not read (their
    // indices clamp to it; nothing past the read's end), and the middle product's bytes past k - 1 read ftab's 1.0.
    auto weight8 = [&](uint64_t qo, uint32_t mask) -> double {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(src.qual + qo);
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)ad & 3u;
        const uint32_t tmax = 31u - (uint32_t)__builtin_clz(mask);  // the last window of the block to weigh
        const uint32_t dl = (sh + k + tmax - 1u) >> 2;                 // the dword of its last byte
        auto ld = [&](uint32_t i) -> uint32_t { return wp[min(i, dl)]; };
        const uint32_t a0 = ld(0), a1 = ld(1), a2 = ld(2);  // bytes 0 .. 7
        const uint32_t rs = sh + k, rd = rs >> 2, rsh = rs & 3u;
        const uint32_t c0 = ld(rd), c1 = ld(rd + 1u), c2 = ld(rd + 2u);  // bytes k .. k + 6
        uint32_t w[5];  // the middle product's first 16 bytes (8 .. 23)
#pragma unroll
        for (uint32_t i = 0; i < 5u; ++i) w[i] = ld(2u + i);
        const uint32_t l03 = __builtin_amdgcn_alignbyte(a1, a0, sh), l47 = __builtin_amdgcn_alignbyte(a2, a1, sh);
        const uint32_t r03 = __builtin_amdgcn_alignbyte(c1, c0, rsh), r47 = __builtin_amdgcn_alignbyte(c2, c1, rsh);
        double S[8];
        S[7] = fac(l47 >> 24);
#pragma unroll
        for (int t = 6; t >= 0; --t) S[t] = fac((t < 4 ? l03 : l47) >> (8 * (t & 3))) * S[t + 1];
        double M = 1.0;
        const uint32_t nbat = (k + 7u) >> 4;  // 16-byte batches of bytes 8 .. k - 1 (uniform)
        auto batch = [&](uint32_t j) {
            uint32_t e[4];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) e[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
            if (j + 1u < nbat) {  // the next 16 bytes' dwords, before this batch's factors
                w[0] = w[4];
#pragma unroll
                for (uint32_t i = 1; i < 5u; ++i) w[i] = ld(6u + 4u * j + i);
            }
            // 16 factors (HW = 4, whose other state holds more registers: two groups of 8, no spills)
            constexpr uint32_t NF = HW >= 4 ? 8u : 16u;
#pragma unroll
            for (uint32_t g = 0; g < 16u; g += NF) {
                double f[NF];
#pragma unroll
                for (uint32_t i = 0; i < NF; ++i) {
                    const uint32_t b = 8u + 16u * j + g + i;  // (b < k: uniform)
                    f[i] = ftab[b < k ? min((e[(g + i) >> 2] >> (8u * (i & 3u))) & 0xFFu, AX_FONE - 1u) : AX_FONE];
                }
#pragma unroll
                for (uint32_t h = NF / 2u; h >= 1u; h >>= 1)
#pragma unroll
                    for (uint32_t i = 0; i < h; ++i) f[i] = f[i] * f[i + h];
                M *= f[0];
            }
        };
        if constexpr (HW == 1) {  // (k <= 32: at most 2 batches, unrolled)
            if (nbat > 0u) batch(0);
            if (nbat > 1u) batch(1);
        } else {
            for (uint32_t j = 0; j < nbat; ++j) batch(j);
        }
        double sum = 0.0, P = M;
#pragma unroll
        for (uint32_t t = 0; t < 8u; ++t) {
            if (t > 0u) P *= fac((t - 1u < 4u ? r03 : r47) >> (8u * ((t - 1u) & 3u)));
            const double x = fma(S[t], P, sum);  // (a window outside the mask may hold rank 0: inf)
            sum = ((mask >> t) & 1u) ? x : sum;
        }
        if (STATS) s_qb += k + tmax;
        return sum;
    };
    // Phred weight of the window whose first quality byte is src.qual[qo]: a window of one quality takes
    // fm_scanner.cpp:454's quotient from wtab (bit-exact); any other window (k >= 8) is weight8's block of one window,
    // for k < 8 the product of its k reciprocals in order.
    auto weight = [&](uint64_t qo, bool uniform) -> double {
        if (uniform) {
            if (STATS) s_qb += 1u;
            const uint32_t x = src.qual[qo];
            return wtab[x < 33u ? 0u : min(x - 33u, 41u)];
        }
        if (k >= 8u) return weight8(qo, 1u);
        double x = 1.0;
        for (uint32_t i = 0; i < k; ++i) x *= fac(src.qual[qo + i]);
        if (STATS) s_qb += k;
        return x;
    };
    // quality-change bits of slot o over slot positions [x, x + len) all zero (local mode)
    auto chg_zero = [&](uint32_t o, uint32_t x, uint32_t len) -> bool {
        uint32_t left = len;
        bool u = true;
        while (left) {
            const uint32_t w = x >> 4, sh = x & 15u, span = min(16u - sh, left);
            const uint32_t mk = (1u << span) - 1u;
            u = u && (w >= AX_CHUNKS || (((uint32_t)chg[w * 64u + o] >> sh) & mk) == 0);
            x += span;
            left -= span;
        }
        return u;
    };

    // ---- the lane's unit and piece
    bool has_unit = false;     // working on a unit (until it is finalized)
    bool last_piece = true;    // the current piece is the unit's last
    uint32_t rd = 0;           // current read (index into off; launch_ax keeps n_units < 2^32)
    uint32_t mate = 0, seg = 0, nseg = 0;
    uint64_t rb = 0;           // current read: first base
    uint32_t L = 0, W = 0;     // its length (< 2^32: a read in HBM with its qualities) and windows
    int32_t af = -1, ad = 0;   // ambiguity state of the unit
    bool hasdef = false;       // deferred windows of this lane's piece are in the wave's list
    // ---- the wave's pool (uniform): an equal share of the units, [nu w / NWV, nu (w + 1) / NWV) — contiguous
    // reads (coalesced staging), and every wave gets the same number of units so the waves finish together (a
    // launch-wide counter handing out groups was slower: one contended atomic address; so were groups of 64-256 units
    // dealt round robin, profiles/r03/ax_variants_owner_group.jsonl)
    uint64_t cur = (nu * gw) / NWV;  // next unit
    const uint64_t cur_end = (nu * (gw + 1)) / NWV;
    const uint64_t pool_n = cur_end - cur;  // (PRIO) units of the pool
    // (PRIO) on for pools of SPEQ_AX_PRIO_MIN units or more (a priority step every few refills) and for k > 64; off for
    // the small pools of light scans, which it slows (config 2 k = 21 +3.5 %: their refills then come in step)
    const bool prio_on = pool_n >= (uint64_t)SPEQ_AX_PRIO_MIN || HW >= 3;
    // ---- phase-1 state of the current piece
    uint32_t wend = 0;         // windows of the piece
    uint32_t off0 = 0;         // first base of the piece in the slot
    uint64_t ta = 0;           // first base of the piece in seq/qual (local mode; other lanes read it by a shuffle)
    uint32_t j = 0;
    uint32_t st = 2u;          // 0: look window j up, 1: extend from text position p, 2: idle, 3: wait for the
                               // deferred-window pass (its deferral found the list full), then look window j up,
                               // 4: window j is absent and the windows [j + 1, last_mm] share its mismatch last_mm:
                               // probe the m-mers over it, defer the windows no absent m-mer covers (MPROOF),
                               // 5: the same for the windows [j, last_mm] of a speculative run, which then resumes,
                               // 6: window j is absent, its mismatch unknown: m-mer probes spread over window j
    bool verify = false;       // st 1: p came from the anchor table (window j itself not compared yet)
    uint32_t p = 0;            // text position of window j (st 1)
    uint32_t gt = 0;           // group of p's text (st 1)
    int32_t last_mm = -1;      // base (relative to the piece) of the last observed mismatch
    uint32_t pb = 0, ps = 0;   // probe position of the current lookup (bucket, first slot)
    bool resume = false;       // continue the current lookup at (pb, ps): full bucket, or failed verification
    bool run_phase = true;     // this wave iteration extends runs (else: looks windows up)
    // Speculative left runs (SPEC, k > 64): a window absent with no known mismatch (the read's first windows over a
    // sequencing error) used to defer the k - 1 windows after it, of which those right of the error are present
    // (each then passes the Bloom filter and costs a phase-2 lookup: ~k/2 per such read, the bulk of the deferred-
    // window pass at k = 70). Instead the lane keeps them pending (sp), looks up the window past them, and on a hit
    // runs from sp against the text shifted back by the pending windows (ps = AX_PS_SPEC): the first mismatch e (the
    // error, which lies in the window before sp) defers only the windows [sp, sp + e] that hold it, and the rest
    // goes on as a run whose first k bases are still to be compared (ps = AX_PS_FRESH). A speculative run must stay in
    // its anchor's text: an END window among the pending ones defers them instead.
    constexpr bool SPEC = HW >= SPEQ_AX_SPEC_HW && !EM && MODE == KM_LOCAL;
    constexpr uint32_t AX_PS_SPEC = 16u, AX_PS_FRESH = 17u;
    // (state 6, unknown mismatches, where no speculative run finds them: compiled into those instantiations only —
    // in the speculative ones its code alone cost k = 70 local 31 %, profiles/r05/ab_mtiles_codegen.jsonl)
    constexpr bool MTILES = SPEQ_AX_MTILES && !SPEC;
    uint32_t sp = 0;  // pending windows [sp, sp + k - 2] of the piece; 0: none
    // defers the valid windows of [lo, hi] (hi - lo <= 127; hi < lo: none) of this lane's piece; when the list has
    // no room: the reserved slots are voided, the lane waits for the deferred-window pass (st 3) and false
    auto defer_except = [&](uint32_t lo, uint32_t hi, uint64_t x0, uint64_t x1) -> bool {  // (x: windows lo + i
        if (hi + 1u <= lo) return true;                                                    // proven absent)
        const uint32_t span = hi + 1u - lo;
        uint64_t dm0 = vbits(lane, lo) & ~x0, dm1 = span > 64u ? (vbits(lane, lo + 64u) & ~x1) : 0ull;
        dm0 &= span >= 64u ? ~0ull : ((1ull << span) - 1ull);
        if (span > 64u) dm1 &= span - 64u >= 64u ? ~0ull : ((1ull << (span - 64u)) - 1ull);
        const uint32_t cnt = (uint32_t)__popcll(dm0) + (uint32_t)__popcll(dm1);
        if (cnt == 0u) return true;
        const uint32_t slot0 = atomicAdd(&defn[0], cnt);
        if (slot0 + cnt > AX_DEF) {
            for (uint32_t sl = slot0; sl < AX_DEF && sl < slot0 + cnt; ++sl) defl[sl] = AX_VOID;
            st = 3u;
            hasdef = true;
            return false;
        }
        uint32_t sl = slot0;
        for (uint64_t t = dm0; t; t &= t - 1) defl[sl++] = (uint16_t)(lane | ((lo + (uint32_t)__builtin_ctzll(t)) << 6));
        for (uint64_t t = dm1; t; t &= t - 1)
            defl[sl++] = (uint16_t)(lane | ((lo + 64u + (uint32_t)__builtin_ctzll(t)) << 6));
        hasdef = true;
        if (STATS) s_def += cnt;
        return true;
    };
    auto defer_range = [&](uint32_t lo, uint32_t hi) -> bool { return defer_except(lo, hi, 0ull, 0ull); };

    auto start_read_at = [&](uint64_t r, uint64_t b, uint64_t e) {  // read r spans [b, e) of seq / qual
        rd = (uint32_t)r;
        rb = b;
        L = (uint32_t)(e - b);
        W = L >= k ? L - k + 1 : 0;
        nseg = W ? (uint32_t)((W + segw - 1) / segw) : 1u;
        seg = 0;
    };
    auto start_read = [&](uint64_t r) { start_read_at(r, src.off[r], src.off[r + 1]); };
    // (PAIRED) the second mate's length, loaded with the first mate's offsets: the second mate then starts at the
    // first's end without another offsets round trip in its refill
    uint32_t L2m = 0;

    // ---- staging of a refill group: the refilling lanes' pieces laid end to end as one stream of 16-base chunks
    // (lane o's at [stg_pre_o, stg_pre_o + stg_nch_o)); every lane of the wave loads and decodes whole chunks, SU x 64
    // chunks per batch, into the owners' slots, one round trip per batch while the wave waits. (Round 6 tried the
    // batches beside the following phase-1 iterations' loads instead: 37 % slower)
    constexpr uint32_t SU = ax_su<MODE, PAIRED, HW>();  // stream instructions of one batch
    static_assert(64u * SU <= ax_ownb<MODE>(), "owner map of one batch");
    static_assert(AX_CHUNKS < 16, "chunk counts in four bits");
    uint32_t stg_tot = 0;      // (wave-uniform) the group's chunks
    uint32_t stg_ocarry = 0;   // (wave-uniform) owner mark of the last chunk of the previous 64
    uint32_t stg_qcarry = 0;   // (wave-uniform, local) last quality dword of the previous instruction's lane 63
    uint32_t stg_pre = 0, stg_nch = 0;  // this lane's piece: first chunk in the group's stream, chunks (0: none)
    // owners and loads of the batch from chunk c0: every refilling lane marks the first chunk of its range in a byte
    // map (lane + 1); a prefix max over the lanes (DPP; owners grow with the chunk index) spreads the mark over the
    // range, and the last owner carries into the next 64 chunks. dst[u] = the owner's slot word (ci * 64 + owner).
    auto stage_issue = [&](uint32_t c0, uint4(&sv)[SU], uint4(&qv)[SU], uint32_t(&dst)[SU]) {
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) ownb[64u * u + lane] = 0;
        if (stg_nch != 0u && stg_pre >= c0 && stg_pre < c0 + 64u * SU) ownb[stg_pre - c0] = (uint8_t)(lane + 1u);
        wave_sync();
        uint32_t mk[SU];
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) mk[u] = ownb[64u * u + lane];
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) {
            const uint32_t c = min(c0 + 64u * u + lane, stg_tot - 1u);
            uint32_t m = mk[u];
            m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x111, 0xF, 0xF, false));  // row_shr:1
            m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x112, 0xF, 0xF, false));  // row_shr:2
            m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x114, 0xF, 0xF, false));  // row_shr:4
            m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x118, 0xF, 0xF, false));  // row_shr:8
            m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x142, 0xA, 0xF, false));  // row_bcast:15
            m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x143, 0xC, 0xF, false));  // row_bcast:31
            m = max(m, stg_ocarry);
            stg_ocarry = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
            const uint32_t o = m - 1u;
            const uint32_t ci = c - (uint32_t)__shfl((int)stg_pre, (int)o);
            dst[u] = ci * 64u + o;
            // the owner's piece starts at ta (its first base); its slot position 0 is ta's 16-B-aligned base
            const uint64_t go = ((uint64_t)__shfl((long long)ta, (int)o) & ~15ull) + 16ull * ci;
            sv[u] = *reinterpret_cast<const uint4*>(src.seq + go);
            qv[u] = *reinterpret_cast<const uint4*>(src.qual + go);
        }
    };
    // decodes the batch from chunk c0 into the owners' slots: 2-bit codes, bad-base bits, quality changes
    auto stage_decode = [&](uint32_t c0, const uint4(&sv)[SU], const uint4(&qv)[SU], const uint32_t(&dst)[SU]) {
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) {
            const uint32_t c = c0 + 64u * u + lane;
            const uint32_t sd[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
            const uint32_t qd[4] = {qv[u].x, qv[u].y, qv[u].z, qv[u].w};
            uint32_t cw = 0, bad = 0, chb = 0;
            // local mode: the quality byte before the chunk (a chunk's change bit 0 compares with it; the piece's
            // first base never reads its change bit)
            uint32_t qprev = 0;
            if (MODE == KM_LOCAL) {  // the previous chunk's last quality (the previous lane's, or the carry)
                const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)qv[u].w, 0x138, 0xF, 0xF, false);
                qprev = lane == 0 ? stg_qcarry : up;
                stg_qcarry = __builtin_amdgcn_readlane(qv[u].w, 63);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t x = sd[i] | 0x20202020u;  // lower case
                const uint32_t c4 = ((x >> 1) ^ (x >> 2)) & 0x03030303u;  // a c g t/u -> 0 1 2 3
                cw |= ((c4 | (c4 >> 6) | (c4 >> 12) | (c4 >> 18)) & 0xFFu) << (8 * i);
                const uint32_t canon = __builtin_amdgcn_perm(0u, 0x74676361u, c4);  // the letter of that code
                const uint32_t okb = zero_bytes(x ^ canon) | zero_bytes(x ^ 0x75757575u);  // ACGT or U
                const uint32_t y = qd[i];
                const uint32_t badq = (((0x80808080u | qt4) - (y & 0x7F7F7F7Fu)) & ~y & 0x80808080u) | allbad;
                bad |= flags4((~okb & 0x80808080u) | badq) << (4 * i);
                if (MODE == KM_LOCAL) {
                    const uint32_t prev = (y << 8) | (qprev >> 24);
                    chb |= flags4(~zero_bytes(y ^ prev) & 0x80808080u) << (4 * i);
                    qprev = y;
                }
            }
            if (c < stg_tot) {
                const uint32_t ci = dst[u] >> 6, o = dst[u] & 63u;
                codes[dst[u]] = cw;
                bad16[((ci >> 2) * 64u + o) * 4u + (ci & 3u)] = (uint16_t)bad;
                if (MODE == KM_LOCAL) chg[dst[u]] = (uint16_t)chb;
            }
        }
    };
    // a staged lane's piece becomes workable: its valid-window bits (from the bad-base bits the decode left in its
    // valid-window words), T, and phase-1 state (the slots' code words were fenced after the decode)
    auto finish_piece = [&](uint32_t nch) {
        // this lane's good-base bits, 16 per chunk from a16 (chunks past its piece are bad), as 8 dwords
        uint32_t ok[8];
        {
            const uint32_t* vw32 = reinterpret_cast<const uint32_t*>(vw);
            const uint32_t nb = 16u * nch;
#pragma unroll
            for (uint32_t d = 0; d < 8u; ++d) {
                const uint32_t b0 = 32u * d;  // dword d: chunks 2d, 2d + 1 (word d / 2 of the lane's column)
                uint32_t v = vw32[((d >> 1) * 64u + lane) * 2u + (d & 1u)];
                v |= nb <= b0 ? ~0u : (nb < b0 + 32u ? ~0u << (nb - b0) : 0u);
                ok[d] = ~v;
            }
        }
        // valid windows: AND of k consecutive good bits (doubling: shifts of at most 64 bits, one funnel shift per
        // dword), then aligned to the piece's first base
        for (uint32_t len = 1u; len < k;) {
            const uint32_t sft = min(len, k - len);  // 1 .. 64
            const uint32_t dw = sft >> 5, bs = sft & 31u;
            if (dw == 0u) {
#pragma unroll
                for (uint32_t d = 0; d < 8u; ++d) ok[d] &= alignbit(d + 1u < 8u ? ok[d + 1] : 0u, ok[d], bs);
            } else if (dw == 1u) {
#pragma unroll
                for (uint32_t d = 0; d < 8u; ++d)
                    ok[d] &= alignbit(d + 2u < 8u ? ok[d + 2] : 0u, d + 1u < 8u ? ok[d + 1] : 0u, bs);
            } else {  // sft == 64
#pragma unroll
                for (uint32_t d = 0; d < 8u; ++d) ok[d] &= d + 2u < 8u ? ok[d + 2] : 0u;
            }
            len += sft;
        }
        // valid-window bits of the piece (window j at bit j): the good-window dwords from slot position off0 (< 16,
        // so dword d + {0, 1}), none past wend (no fence: every lane writes and then reads only its own column)
        {
            uint32_t* vw32 = reinterpret_cast<uint32_t*>(vw);
            uint32_t tc = 0;  // T (fm_scanner.cpp:164): the piece's passing windows
#pragma unroll
            for (uint32_t d = 0; d < 2u * AX_VWW; ++d) {
                uint32_t v = alignbit(d + 1u < 8u ? ok[d + 1] : 0u, ok[d], off0);
                const uint32_t bit0 = 32u * d;
                v = wend <= bit0 ? 0u : (wend < bit0 + 32u ? v & ((1u << (wend - bit0)) - 1u) : v);
                tc += (uint32_t)__popc(v);
                vw32[((d >> 1) * 64u + lane) * 2u + (d & 1u)] = v;
            }
            if (tc) atomicAdd(&wsum[0], (unsigned long long)tc);
        }
        j = 0;
        if (SPEC) sp = 0;
        st = wend > 0 ? 0u : 2u;
        verify = false;
        resume = false;
        last_mm = -1;
    };
    for (;;) {
        // ================= housekeeping (wave-uniform decisions) =================
        const unsigned long long idle = __ballot(st == 2u);
        const unsigned long long blk = __ballot((st == 2u || st == 3u) && hasdef);
        const unsigned long long busy = ~idle;
        // (a lane whose deferral found the list full, st 3, counts as blocked: the list then holds more than AX_DEF
        // entries, so this pass runs, and the lane looks its window up again afterwards)
        const bool p2 = blk != 0 && ((uint32_t)__popcll(blk) >= SPEQ_AX_BLOCKED || busy == 0 ||
                                     (uint32_t)__builtin_amdgcn_readfirstlane(defn[0]) + (uint32_t)SPEQ_AX_P2_MARGIN > AX_DEF);
        // (the list length is read only when the pass runs: an LDS round trip on every iteration's critical path
        // cost 8-10 %, profiles/r03/ax_variants_micro_interleaved_s3.jsonl)
        const uint32_t n_def = p2 ? __builtin_amdgcn_readfirstlane(defn[0]) : 0u;
        if (STATS) c_s = clock64();
        if (p2) {
            // ---- phase 2: the deferred windows of the wave. (a) the Bloom filter, AX_F windows per lane per round
            // trip; the windows it cannot rule out are compacted to the front of the list; (b) those are looked up
            // one per lane (bucket -> fingerprint -> compare with the text -> class)
            ambf[lane] = af;
            ambd[lane] = ad;
            wave_sync();
            const uint32_t n2 = min(n_def, AX_DEF);
            for (uint32_t base = 0; base < n2; base += 64u * AX_F) {
                uint32_t ent[AX_F];
                uint64_t hh[AX_F];
                uint64_t fw[AX_F];
                // in stages over the AX_F entries (entries, then their slot offsets, then their bases), so each stage's
                // LDS reads are in flight together instead of one dependent chain per entry
                uint32_t so[AX_F];
#pragma unroll
                for (uint32_t t = 0; t < AX_F; ++t) {
                    const uint32_t idx = base + 64u * t + lane;
                    const uint16_t e16 = defl[min(idx, AX_DEF - 1u)];
                    ent[t] = (idx < n2 && e16 != AX_VOID) ? (uint32_t)e16 : AX_EMPTY;
                }
#pragma unroll
                for (uint32_t t = 0; t < AX_F; ++t) so[t] = (uint32_t)off0s[ent[t] & 63u] + ((ent[t] >> 6) & 1023u);
#pragma unroll
                for (uint32_t t = 0; t < AX_F; ++t) {
                    uint64_t ra[HW];
                    read_words(ent[t] & 63u, so[t], ra);
                    hh[t] = ax_hash<HW>(ra, k);
                }
#pragma unroll
                for (uint32_t t = 0; t < AX_F; ++t) {
                    const uint32_t foff = ent[t] != AX_EMPTY ? ax_fword(hh[t], A.nf) * 8u : AX_OOB;
                    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_filt, foff, 0, 0);
                    fw[t] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
                }
                wave_sync();  // every lane has read its entries before any survivor overwrites the list's front
#pragma unroll
                for (uint32_t t = 0; t < AX_F; ++t) {
                    const uint64_t bits = ax_fbits(hh[t]);
                    if (ent[t] != AX_EMPTY && (fw[t] & bits) == bits) {
                        const uint32_t slot = atomicAdd(&defn[1], 1u);
                        defl[slot] = (uint16_t)ent[t];
                    }
                }
                wave_sync();
            }
            const uint32_t n3 = __builtin_amdgcn_readfirstlane(defn[1]);
            if (STATS) {
                s_fp += lane == 0 ? n3 : 0u;
                c_p2f += clock64() - c_s;
            }
            for (uint32_t base = 0; base < n3; base += 64) {
                const uint32_t idx = base + lane;
                const bool act = idx < n3;
                const uint32_t ent = act ? (uint32_t)defl[idx] : 0u;
                const uint32_t o = ent & 63u, jj = ent >> 6;
                const uint32_t so = (uint32_t)off0s[o] + jj;  // the window's slot position
                // local mode: the first base of lane o's piece (every lane active here: a full-wave shuffle)
                const uint64_t tao = MODE == KM_LOCAL ? (uint64_t)__shfl((long long)ta, (int)o) : 0ull;
                uint64_t ra[HW];
                read_words(o, so, ra);
                const uint64_t h = ax_hash<HW>(ra, k);
                const uint32_t fp = ax_fp(h);
                uint32_t b = act ? ax_bucket(h, A.nb) : 0u, sl = 0, pp = 0, pg = 0;
                bool pend = act, found = false;
                uint32_t cl = AX_SENT;
                while (__ballot(pend) != 0) {
                    if (STATS) s_p2r += lane == 0 ? 1u : 0u;
                    const bool c = ax_probe(A, rs_atab, fp, b, sl, pp, pg, pend, s_p2);
                    const bool cand = pend && c;
                    if (STATS) s_p2v += cand ? 1u : 0u;
                    u32x4 gv[HW + 1];
                    {
                        const uint32_t goff = cand ? (pp >> 5) * 16u : AX_OOB;
#pragma unroll
                        for (int i = 0; i <= HW; ++i)
                            gv[i] = __builtin_amdgcn_raw_buffer_load_b128(rs_gran, goff + 16u * (uint32_t)i, 0, 0);
                    }
                    if (pend) {
                        if (!c) {
                            pend = false;  // absent
                        } else {
                            const uint32_t s5 = pp & 31u;
                            bool eq = true;
#pragma unroll
                            for (int i = 0; i < HW; ++i) {
                                uint64_t x = ra[i] ^ funnel(u64of(gv[i][0], gv[i][1]), u64of(gv[i + 1][0], gv[i + 1][1]),
                                                            2u * s5);
                                const uint32_t b0 = 32u * (uint32_t)i;
                                if (k <= b0) x = 0;
                                else if (k < b0 + 32u) x &= (1ull << (2u * (k - b0))) - 1ull;
                                eq = eq && x == 0;
                            }
                            if (eq) {
                                found = true;
                                cl = ((gv[0][2] >> s5) & 1u) | (((gv[0][3] >> s5) & 1u) << 1);
                                pend = false;
                            } else {
                                ++sl;  // fingerprint collision: keep probing
                            }
                        }
                    }
                }
                if (found && cl == AX_OWN) {
                    double wgt = 0.0;
                    if (MODE == KM_LOCAL) wgt = weight(tao + jj, chg_zero(o, so + 1u, k - 1u));
                    add_count(pg, 1u, wgt);
                    const int32_t old = atomicCAS(&ambf[o], -1, (int32_t)pg);
                    if (old != -1 && old != (int32_t)pg) ambd[o] = 1;
                } else if (EM && found && cl == AX_MULTI) {
                    const uint32_t lo = A.mlo[pp];
                    atomicAdd(&src.em_mult[lo], 1u);
                    src.em_hi[lo] = A.mhi[lo];
                }
            }
            wave_sync();
            af = ambf[lane];
            ad = ambd[lane];
            hasdef = false;
            st = st == 3u ? 0u : st;  // retry the lookup whose deferral found the list full
            if (lane == 0) defn[0] = defn[1] = 0u;
            wave_sync();
            if (STATS) {
                c_p2 += clock64() - c_s;
                s_p2n += lane == 0 ? 1u : 0u;
            }
            continue;
        }
        // lanes that can start a piece now: idle, no deferred windows pending, and a next piece of their unit or
        // a unit left in the pool
        const bool ready = st == 2u && !hasdef;
        const bool more_pool = cur < cur_end;
        const bool wants = ready && ((has_unit && !last_piece) || more_pool);
        const unsigned long long want = __ballot(wants);
        if (want == 0 && busy == 0) {
            if (blk == 0) break;  // (blk != 0 with busy == 0 ran phase 2 above)
        }
        if (want != 0 && ((uint32_t)__popcll(want) >= SPEQ_AX_REFILL || busy == 0)) {
            // ================= refill: next pieces of the wanting lanes, staged together =================
            if (STATS) s_spl += lane == 0 ? 1u : 0u;
            if (wants && has_unit && last_piece) {  // the unit is complete: its ambiguity (fm_scanner.cpp:183-190)
                if (ad) atomicAdd(&wsum[1], 1ull);
                has_unit = false;
                af = -1;
                ad = 0;
            }
            // units from the pool for the lanes without one, in lane order
            const unsigned long long tk = __ballot(wants && !has_unit);
            uint64_t newu = nu;
            const uint32_t rank = lanes_below(tk);
            const uint64_t taken = (uint64_t)__popcll(tk);
            if (wants && !has_unit && cur + rank < cur_end) newu = cur + rank;
            cur = min(cur + taken, cur_end);
            if (SPEQ_AX_PRIO && prio_on) {
                // issue priority by the share of the pool still to do: the SIMD's arbiter favours the oldest wave at
                // equal priority, so without this the waves dispatched first finish in a third of the time of the
                // last ones and the SIMD runs the end of the launch with few waves (profiles/r04/stats_gen.jsonl)
                const uint32_t q = (uint32_t)(((cur_end - cur) * 4u) / (pool_n + 1u));
                if (q >= 3u) __builtin_amdgcn_s_setprio(3);
                else if (q == 2u) __builtin_amdgcn_s_setprio(2);
                else if (q == 1u) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
            bool stg = false;
            if (wants) {
                if (!has_unit) {
                    if (newu < nu) {
                        has_unit = true;
                        mate = 0;
                        if (PAIRED) {
                            const uint64_t r0 = 2 * newu, o0 = src.off[r0], o1 = src.off[r0 + 1], o2 = src.off[r0 + 2];
                            start_read_at(r0, o0, o1);
                            L2m = (uint32_t)(o2 - o1);
                        } else {
                            start_read(newu);
                        }
                        stg = true;
                    }
                } else if (seg + 1u < nseg) {
                    ++seg;
                    stg = true;
                } else {  // PAIRED: the second mate
                    mate = 1;
                    start_read_at(rd + 1, rb + L, rb + L + L2m);
                    stg = true;
                }
            }
            // the piece: bases [s, s + sb), windows [s, s + wend) of read rd
            const uint64_t s = (uint64_t)seg * segw;
            const uint32_t sb = stg && W ? (uint32_t)(L - s < AX_CAP ? L - s : AX_CAP) : 0u;
            const uint32_t nwend = stg && W ? (uint32_t)(W - s < segw ? W - s : segw) : 0u;  // (s < W here)
            const uint64_t a = rb + s;
            const uint64_t a16 = a & ~15ull;
            const uint32_t noff0 = (uint32_t)(a - a16);
            const uint32_t nch = sb ? (noff0 + sb + 15u) / 16u : 0u;
            if (stg) {
                last_piece = seg + 1u >= nseg && (!PAIRED || mate == 1u);
                wend = nwend;
                off0 = noff0;
                ta = a;
                off0s[lane] = (uint8_t)noff0;
                if (STATS) {
                    s_ch += nch;
                    s_seg += 1u;
                }
            }
            // ---- the group's chunk stream: lane o's chunks at [pre_o, pre_o + nch_o)
            uint32_t pre = 0, nch_tot = 0;
#pragma unroll
            for (uint32_t bb = 0; bb < 4; ++bb) {
                const unsigned long long m = __ballot((nch >> bb) & 1u);
                pre += lanes_below(m) << bb;
                nch_tot += (uint32_t)__popcll(m) << bb;
            }
            stg_pre = pre;
            stg_nch = stg ? nch : 0u;
            stg_tot = nch_tot;
            stg_ocarry = 0;
            stg_qcarry = 0;
            uint64_t c_b = 0;
            if (STATS) {
                c_b = clock64();
                c_rpre += c_b - c_s;
            }
            for (uint32_t c0 = 0; c0 < nch_tot; c0 += 64u * SU) {
                uint4 sv[SU], qv[SU];
                uint32_t dst[SU];
                stage_issue(c0, sv, qv, dst);
                stage_decode(c0, sv, qv, dst);
            }
            wave_sync();
            if (STATS) c_rstg += clock64() - c_b;
            if (stg) finish_piece(nch);
            // the slots' code words were fenced after the decode (phase 2 reads other lanes' slots); the valid-window
            // bits are read by their own lane only
            if (STATS) c_ref += clock64() - c_s;
            continue;  // re-evaluate (lanes whose piece has no window are idle again)
        }
        if (busy == 0) continue;  // blocked lanes only: phase 2 runs next time round

        // ================= phase 1: one memory round trip per iteration =================
        // a lane either probes the anchor table (its candidate is compared in the next iteration) or extends a run
        // over the rest of its piece (at most AX_CMP bases; a clean 150-bp read: one lookup and one run). One kind
        // of work per iteration, alternating (a lookup is followed by a run and a run by a lookup, so a lane rarely
        // waits): the wave executes the lookup code or the run code, not both under exec masks (the kernel is bound
        // by VALU issue, profiles/r03), and a kind no lane needs is skipped.
        // the next valid window of a lane waiting to look one up is found in the lookup iteration itself, so a run
        // iteration does not wait for those lanes' LDS reads; such a lane may count as busy one iteration longer
        const unsigned long long busy1 = __ballot(st != 2u);
        if (busy1 == 0) continue;
        if (STATS && lane == 0) {
            const uint32_t nb = (uint32_t)__popcll(busy1);
            s_b4 += nb <= 4u ? 1u : 0u;
            s_b16 += (nb > 4u && nb <= 16u) ? 1u : 0u;
            s_b32 += (nb > 16u && nb <= 32u) ? 1u : 0u;
            s_b64 += nb > 32u ? 1u : 0u;
        }
        const bool want_lk = __ballot(st == 0u || st >= 4u) != 0, want_rn = __ballot(st == 1u) != 0;
        run_phase = run_phase ? !want_lk : want_rn;
        // lookup iterations: the window's code words are read together with its valid bits (the same
        // window unless it is not valid, then read again), one LDS round trip before the bucket load instead of two
        // (single-end k <= 32 only: elsewhere the words held across the valid-bit search spill)
        constexpr bool SPEC_RW = HW == 1 && !PAIRED;
        uint64_t ra[HW];
        if (!run_phase && st == 0u) {
            const uint32_t j0 = j;
            if (SPEC_RW) read_words(lane, off0 + j0, ra);
            j = next_valid(lane, j0, wend);
            if (SPEC && sp != 0u && j >= wend && defer_range(sp, min(sp + k - 2u, wend - 1u)))
                sp = 0;  // no window left to anchor the pending ones (no room: st 3, kept)
            if (j >= wend && st == 0u) st = 2u;
            else if (SPEC_RW && j != j0) read_words(lane, off0 + j, ra);
        }
        const bool lk = st == 0u && !run_phase, rn = st == 1u && run_phase;
        if (STATS) {
            s_iter += lane == 0 ? 1u : 0u;
            s_lkw += (lane == 0 && !run_phase) ? 1u : 0u;
            s_rnw += (lane == 0 && run_phase) ? 1u : 0u;
            s_lk += lk ? 1u : 0u;
            s_rn += rn ? 1u : 0u;
        }
        if (!run_phase) {
            // ---- lookup: hash window j -> bucket (8 slots {pos, fp | group}); resolve
            if (!SPEC_RW) read_words(lane, off0 + j, ra);
            const uint64_t h = ax_hash<HW>(ra, k);
            const uint32_t fp = ax_fp(h);
            if (lk && !resume) {
                pb = ax_bucket(h, A.nb);
                ps = 0;
            }
            // the 64-B bucket pb of the probe chain
            const uint32_t boff = lk ? pb * 64u : AX_OOB;
            uint32_t o0 = boff, o1 = lk ? boff + 16u : AX_OOB, o2 = lk ? boff + 32u : AX_OOB,
                     o3 = lk ? boff + 48u : AX_OOB;
            // (MPROOF, state 4) the windows lo .. hi (lo = j + 1, hi = min(e, wend - 1)) all contain the mismatch
            // e = last_mm. Probe t tests the m-mer from read base a_t (a_0 = min(e, lo + k - m), then steps of
            // k - m + 1, at most e: every probe's m-mer holds e); it lies inside the windows a_t - (k - m) .. a_t, so
            // when its filter bits are missing those windows are absent. The probes' filter words are loaded by the
            // same four instructions as a bucket (lanes in state 4 never load one); mb[t]: bit indices, bit 31 = used
            // (state 5: the windows j .. e of a speculative run, lo = j, then the run resumes)
            const bool mk = SPEQ_AX_MPROOF && st >= 4u;
            const uint32_t km = k - A.m;
            uint32_t mb[AX_MP] = {0u, 0u, 0u, 0u};
            static_assert(AX_MP == 4, "one m-mer probe per bucket load");
            // (state 6: window j is absent with no known mismatch: np m-mers spread evenly over window j's bases
            // locate the error: the last absent one, at a_R, proves the windows that contain it and the windows up to
            // a_R + m - 1 are deferred, the later ones looked up as usual)
            const bool tiles = MTILES && st == 6u;
            if (SPEQ_AX_MPROOF && mk) {
                const uint32_t e = tiles ? 0u : (uint32_t)last_mm;
                const uint32_t np = tiles ? min(AX_MP, (k + A.m - 1u) / A.m) : AX_MP;  // (tiles: >= 2, k > m)
                uint32_t a = tiles ? j : min(e, j + (st == 4u ? 1u : 0u) + km);
#pragma unroll
                for (uint32_t t = 0; t < AX_MP; ++t) {
                    if (tiles) {
                        if (t >= np) break;
                        a = j + (t * km) / (np - 1u);
                    }
                    const uint64_t x[1] = {slot64(lane, off0 + a)};
                    const uint64_t hm = ax_hash<1>(x, A.m);
                    const uint32_t off = A.mf_off + ax_fword(hm, A.nmf) * 8u;
                    mb[t] = 0x80000000u | ((uint32_t)hm & 0x3FFFFu) | (a << 18);
                    if (t == 0u) o0 = off;
                    else if (t == 1u) o1 = off;
                    else if (t == 2u) o2 = off;
                    else o3 = off;
                    if (!tiles) {
                        if (a == e) break;  // (the last probe: later ones stay unused)
                        a = min(e, a + km + 1u);
                    }
                }
            }
            const u32x4 q0 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, o0, 0, 0);
            const u32x4 q1 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, o1, 0, 0);
            const u32x4 q2 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, o2, 0, 0);
            const u32x4 q3 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, o3, 0, 0);

            if (SPEQ_AX_MPROOF && mk) {
                // windows proven absent, relative to lo (at most k - 1 <= 127 of them): two 64-bit masks
                const uint32_t lo = j + (st == 5u ? 0u : 1u);
                uint32_t hi = min(tiles ? j + k - 1u : (uint32_t)last_mm, wend - 1u);
                uint64_t x0 = 0, x1 = 0;
                uint32_t aR = 0;  // (tiles) 1 + the last absent m-mer's start

                const u32x4 qv[AX_MP] = {q0, q1, q2, q3};
#pragma unroll
                for (uint32_t t = 0; t < AX_MP; ++t) {
                    if (!(mb[t] >> 31)) continue;
                    const uint64_t word = (uint64_t)qv[t][0] | ((uint64_t)qv[t][1] << 32);
                    const uint64_t bits = ax_fbits((uint64_t)(mb[t] & 0x3FFFFu));
                    if ((word & bits) == bits) continue;  // the m-mer may occur: its windows stay deferred
                    const uint32_t a = (mb[t] >> 18) & 0x1FFFu;
                    aR = max(aR, a + 1u);
                    if (a < lo) continue;  // (tile 0 at window j: it only locates the error)
                    const uint32_t r0 = (a >= lo + km ? a - km : lo) - lo, r1 = min(a, hi) - lo;  // covered lo + r0 ..
                    // bits r0 .. r1 of the 128-bit mask x1:x0
                    const uint64_t m0 = r0 >= 64u ? 0ull : (~0ull << r0) & (r1 >= 63u ? ~0ull : ((2ull << r1) - 1ull));
                    const uint64_t m1 = r1 < 64u ? 0ull
                                                 : ((r0 <= 64u ? ~0ull : (~0ull << (r0 - 64u))) &
                                                    (r1 - 64u >= 63u ? ~0ull : ((2ull << (r1 - 64u)) - 1ull)));
                    x0 |= m0;
                    x1 |= m1;
                }
                if (tiles && aR != 0u) hi = min(aR - 1u + A.m - 1u, hi);  // later windows: looked up as usual
                const bool resume_run = st == 5u;
                st = 0u;
                if (defer_except(lo, hi, x0, x1)) {  // (no room: st 3, and window j is looked up again afterwards)
                    if (SPEC && resume_run) {  // the speculative run goes on after the mismatch, fresh
                        p += hi + 1u - j;
                        ps = AX_PS_FRESH;
                        st = hi + 1u < wend ? 1u : 2u;
                    }
                    j = hi + 1u;
                    last_mm = -1;
                } else if (SPEC && resume_run) {  // (state 4 keeps last_mm: the retried lookup probes again)
                    ps = 0;
                    resume = false;
                    last_mm = -1;
                }
            }
            if (lk) {
                uint32_t slot = 0, cp = 0, cg = 0;
                const uint32_t res = ax_resolve(q0, q1, q2, q3, fp, ps, slot, cp, cg);
                if (res == 1u) {  // candidate: compared with the text in the next iteration
                    p = cp;
                    gt = cg;
                    ps = slot;
                    st = 1u;
                    verify = true;
                    resume = false;
                    if (SPEC && sp != 0u) {  // pending windows [sp, j): the run starts there, text shifted back
                        const uint32_t back = j - sp;
                        if (cp >= back) {
                            p = cp - back;
                            j = sp;
                            ps = AX_PS_SPEC;
                            pb = back;  // (no probe to resume from a speculative run)
                            sp = 0;
                        } else if (defer_range(sp, j - 1u)) {  // (the text's start) defer them
                            sp = 0;
                        }  // (no room: st 3, the lookup is redone after the deferred-window pass)
                    }
                } else if (res == 0u) {
                    // absent: defer the windows that share the mismatch (or the next k - 1), skip past them; (SPEC)
                    // mismatch unknown: keep the next k - 1 windows pending and look up the one after them
                    resume = false;
                    const bool known = last_mm >= (int32_t)j && last_mm < (int32_t)(j + k);
                    if (SPEC && !known && j + k < wend) {
                        if (sp == 0u || defer_range(sp, sp + k - 2u)) {  // (an earlier pending range first)
                            sp = j + 1u;
                            j += k;
                            last_mm = -1;
                        }
                    } else if (!SPEC || sp == 0u || defer_range(sp, min(sp + k - 2u, j - 1u))) {
                        if (SPEC) sp = 0;
                        uint32_t dend = known ? (uint32_t)last_mm : j + k - 1u;
                        dend = min(dend, wend - 1u);
                        // (no room: the lane waits for the deferred-window pass, st 3, and looks window j up again
                        // afterwards — one wasted lookup instead of looking up all k - 1 windows one by one)
                        if (SPEQ_AX_MPROOF && A.m != 0u && dend > j) {
                            st = known ? 4u : ((MTILES && A.mtiles) ? 6u : 0u);  // probes next lookup
                            if (st == 0u && defer_range(j + 1u, dend)) {
                                j = dend + 1u;
                                last_mm = -1;
                            }
                        } else if (defer_range(j + 1u, dend)) {
                            j = dend + 1u;
                            last_mm = -1;
                        }
                    }
                } else {  // full bucket without the key or an empty slot: the next bucket
                    pb = pb + 1u == (uint32_t)A.nb ? 0u : pb + 1u;
                    ps = 0;
                    resume = true;
                }
            }
        } else {
            // ---- run: compare read [j, j + cl) with text [p, p + cl) (cl = the rest of the piece, at most AX_CMP
            // bases: the granules that cover it from p's granule on, the others with out-of-range offsets), then
            // classify the matched windows
            const uint32_t cl = min(wend - j + k - 1u, AX_CMP);
            const uint32_t ng = rn ? ((p & 31u) + cl + 31u) >> 5 : 0u;
            const uint32_t goff = (p >> 5) * 16u;
            u32x4 gr[AX_NGR];
#pragma unroll
            for (uint32_t i = 0; i < AX_NGR; ++i)
                gr[i] = __builtin_amdgcn_raw_buffer_load_b128(rs_gran, i < ng ? goff + 16u * i : AX_OOB, 0, 0);

            if (STATS) s_rg += ng;
            uint32_t qj = 0;
            if (MODE == KM_LOCAL) {
                qj = src.qual[ta + (rn ? j : 0u)];
                if (STATS) s_qb += rn ? 1u : 0u;
            }
            // the read's 16-base dwords from slot position off0 + j
            const uint32_t rpos = off0 + j, rd0 = rpos >> 4, rsh = 2u * (rpos & 15u);
            uint32_t rw[AX_CMPW * 2 + 1];
#pragma unroll
            for (uint32_t i = 0; i <= 2 * AX_CMPW; ++i) {
                const uint32_t d = rd0 + i;
                rw[i] = d < AX_CHUNKS ? codes[d * 64u + lane] : 0u;
            }
            // a run's own windows (chunk c: windows j + 32 c ..); with varying qualities (local mode), weighed by
            // the whole wave after the run (wl_pend; run group wl_g, first window wl_j)
            uint32_t ownc[AX_CMPW] = {0u, 0u, 0u, 0u, 0u};
            static_assert(AX_CMPW == 5, "five 32-window chunks");
            bool wl_pend = false;
            uint32_t wl_g = 0, wl_j = 0;
            if (rn) {
                const uint32_t s5 = p & 31u, q16 = s5 >> 4, tsh = 2u * (s5 & 15u);
                uint32_t e = cl;  // first mismatching base (cl: none)
#pragma unroll
                for (int i = 2 * (int)AX_CMPW - 1; i >= 0; --i) {
                    // text dwords T[m] = gr[m / 2][m % 2]; aligned: bases 16 i .. 16 i + 15 from p
                    const uint32_t m0 = (uint32_t)i, m1 = (uint32_t)i + 1u, m2 = (uint32_t)i + 2u;
                    const uint32_t t0 = gr[m0 / 2][m0 % 2], t1 = gr[m1 / 2][m1 % 2];
                    const uint32_t t2 = m2 / 2 < AX_NGR ? gr[(m2 / 2) % AX_NGR][m2 % 2] : 0u;
                    const uint32_t tlo = q16 ? t1 : t0, thi = q16 ? t2 : t1;
                    const uint32_t td = alignbit(thi, tlo, tsh);
                    const uint32_t rdw = alignbit(rw[i + 1], rw[i], rsh);
                    uint32_t x = td ^ rdw;
                    const uint32_t b0 = 16u * (uint32_t)i;
                    e = x ? b0 + ((uint32_t)__builtin_ctz(x) >> 1) : e;
                }
                // bases past cl compare whatever lies there (zeros past the staged chunks and the loaded
                // granules): a mismatch among them only matters as "none before cl"
                e = min(e, cl);
                // (SPEC) a speculative run must stay in its anchor's text: an END window (a text end) among the pending
                // windows [0, pb) defers them, and the anchored window is compared from its own position next
                bool sep = false;
                if (SPEC && ps == AX_PS_SPEC) {
#pragma unroll
                    for (uint32_t c = 0; c < 4u; ++c) {
                        const uint32_t w0 = 32u * c;
                        const uint32_t P0 = alignbit(gr[c + 1][2], gr[c][2], s5);
                        const uint32_t P1 = alignbit(gr[c + 1][3], gr[c][3], s5);
                        const uint32_t m = pb <= w0 ? 0u : (pb - w0 >= 32u ? ~0u : ((1u << (pb - w0)) - 1u));
                        sep = sep || (P0 & P1 & m) != 0u;
                    }
                }
                if (SPEC && sep) {
                    if (defer_range(j, j + pb - 1u)) {
                        j += pb;
                        p += pb;
                        ps = AX_PS_FRESH;  // (verify stays set)
                    } else {
                        ps = 0;  // no room (st 3): window j is looked up after the deferred-window pass
                        resume = false;
                    }
                    last_mm = -1;
                } else if (SPEC && verify && e < k && ps == AX_PS_SPEC) {
                    // the windows [j, j + e] hold the speculative run's first mismatch (the read's error): deferred;
                    // the run goes on after it, its first k bases still to be compared. (MPROOF: state 5 first proves
                    // them absent by m-mer probes over base j + e where it can, then resumes this run)
                    if (SPEQ_AX_MPROOF && A.m != 0u && j + e < wend) {
                        last_mm = (int32_t)(j + e);
                        st = 5u;
                    } else {
                        if (defer_range(j, j + e)) {
                            j += e + 1u;
                            p += e + 1u;
                            ps = AX_PS_FRESH;
                            st = j < wend ? 1u : 2u;
                        } else {
                            ps = 0;
                            resume = false;
                        }
                        last_mm = -1;
                    }
                } else if (SPEC && verify && e < k && ps == AX_PS_FRESH) {  // no match from here: look window j up
                    st = 0u;
                    resume = false;
                    ps = 0;
                    last_mm = (int32_t)(j + e);
                } else if (verify && e < k) {  // fingerprint collision: resume probing after that slot
                    st = 0u;
                    resume = true;
                    ++ps;
                } else {
                    uint32_t R = e - (k - 1u);  // e >= k - 1: a candidate matched k bases, a run k - 1
                    R = min(R, wend - j);
                    // the windows [0, R) in 32-window chunks: class planes of windows p + 32c .. (bits s5 + 32c ..
                    // of the granules' planes). The run stops at the first END window (the text ends: the next
                    // windows belong to another text, looked up again) or SENT window of a valid read window (an N
                    // in the text: looked up); windows before it are tallied to the run's group.
                    uint32_t d0 = R, cnt = 0;
                    bool cut = false, cut_end = false;
                    // the lane's valid-window bits j .. j + 159 as 32-bit chunks (dwords of its vw column)
                    uint32_t vm[AX_CMPW];
                    {
                        const uint32_t* vw32 = reinterpret_cast<const uint32_t*>(vw);
                        const uint32_t d = j >> 5, vs = j & 31u;
                        uint32_t vd[AX_CMPW + 1];
#pragma unroll
                        for (uint32_t i = 0; i <= AX_CMPW; ++i) {
                            const uint32_t di = d + i;
                            vd[i] = di < 2u * AX_VWW ? vw32[((di >> 1) * 64u + lane) * 2u + (di & 1u)] : 0u;
                        }
#pragma unroll
                        for (uint32_t i = 0; i < AX_CMPW; ++i) vm[i] = alignbit(vd[i + 1], vd[i], vs);
                    }
                    // windows of chunk c in the run (none past R)
                    auto run_mask = [&](uint32_t c) -> uint32_t {
                        const uint32_t w0 = 32u * c;
                        return R <= w0 ? 0u : (R - w0 >= 32u ? ~0u : ((1u << (R - w0)) - 1u));
                    };
                    // common case first: no END / SENT window in the run (no stop): the tally is one popcount per
                    // chunk; runs with a stop (rare) are recounted below with the windows before it only
                    uint32_t anystop = 0;
                    if (!EM) {
#pragma unroll
                        for (uint32_t c = 0; c < AX_CMPW; ++c) {
                            if (c > 0 && __ballot(R > 32u * c) == 0) break;
                            const uint32_t mR = run_mask(c);
                            const uint32_t P0 = alignbit(gr[c + 1][2], gr[c][2], s5);
                            const uint32_t P1 = alignbit(gr[c + 1][3], gr[c][3], s5);
                            const uint32_t m = vm[c] & mR;
                            anystop |= P1 & (P0 | m) & mR;
                            const uint32_t ow = ~(P0 | P1) & m;
                            cnt += (uint32_t)__popc(ow);
                            ownc[c] = ow;
                        }
                    }
                    if (EM || __ballot(anystop != 0) != 0) {
                        if (EM || anystop != 0) {
                            cnt = 0;
#pragma unroll
                            for (uint32_t c = 0; c < AX_CMPW; ++c) {
                                const uint32_t w0 = 32u * c;
                                const uint32_t mR = run_mask(c);
                                const uint32_t P0 = alignbit(gr[c + 1][2], gr[c][2], s5);
                                const uint32_t P1 = alignbit(gr[c + 1][3], gr[c][3], s5);
                                const uint32_t m = vm[c] & mR;  // the chunk's valid read windows in the run
                                const uint32_t stop = P1 & (P0 | m) & mR;
                                const uint32_t below = cut ? 0u : (stop ? ((stop & (0u - stop)) - 1u) : ~0u);
                                const uint32_t ow = ~(P0 | P1) & m & below;
                                cnt += (uint32_t)__popc(ow);
                                ownc[c] = ow;
                                if (EM) {  // multi-group windows of the run: the EM histogram
                                    uint32_t todo = P0 & ~P1 & m & below;
                                    while (todo) {
                                        const uint32_t d = (uint32_t)__builtin_ctz(todo);
                                        todo &= todo - 1;
                                        const uint32_t lo = A.mlo[p + w0 + d];
                                        atomicAdd(&src.em_mult[lo], 1u);
                                        src.em_hi[lo] = A.mhi[lo];
                                    }
                                }
                                if (!cut && stop) {
                                    const uint32_t t = (uint32_t)__builtin_ctz(stop);
                                    d0 = w0 + t;
                                    cut_end = ((P0 >> t) & 1u) != 0;
                                    cut = true;
                                }
                            }
                        }
                    }
                    if (STATS) {
                        s_rwin += d0;
                        s_tal += cnt;
                    }
                    if (cnt) {
                        double wsum = 0.0;
                        if (MODE == KM_LOCAL) {
                            // one quality for the whole cut run when no base in (j, j + d0 - 1 + k) changes it
                            if (chg_zero(lane, rpos + 1u, d0 + k - 2u)) {
                                int q = (int)qj - 33;
                                q = q < 0 ? 0 : (q > 41 ? 41 : q);
                                wsum = (double)cnt * wtab[q];
                            } else {
                                wl_pend = true;
                                wl_g = gt;
                                wl_j = j;
                            }
                        }
                        add_count(gt, cnt, wsum);
                        if (af < 0) af = (int32_t)gt;
                        else if ((int32_t)gt != af) ad = 1;
                    }
                    // next state
                    verify = false;
                    if (d0 < R) {
                        if (cut_end) {  // END: look the window up (its k-mer may occur elsewhere)
                            j += d0;
                            st = 0u;
                            resume = false;
                            last_mm = -1;
                        } else {  // SENT: matched bases, but no valid text window: deferred (or looked up now)
                            const uint32_t slot = atomicAdd(&defn[0], 1u);
                            if (slot < AX_DEF) {
                                defl[slot] = (uint16_t)(lane | ((j + d0) << 6));
                                hasdef = true;
                                if (STATS) s_def += 1u;
                                j += d0 + 1u;
                                p += d0 + 1u;
                                st = 1u;
                            } else {
                                j += d0;
                                st = 0u;
                                resume = false;
                                last_mm = -1;
                            }
                        }
                    } else {
                        const bool mism = e < cl;  // the run ended at a mismatch (base j + e)
                        if (mism && R < wend - j) last_mm = (int32_t)(j + e);
                        j += R;
                        p += R;
                        st = (mism || R == 0u) ? 0u : 1u;
                        if (st == 0u) resume = false;
                    }
                    if (j >= wend) st = 2u;
                }
            }
            if (MODE == KM_LOCAL && __ballot(wl_pend) != 0) {
                // runs with varying qualities: their own windows in 8-window blocks (20 per run), weighed by the
                // whole wave, every lane's blocks at once: each lane writes its blocks' entries at its prefix of the
                // wave's block counts, AX_WL entries per round, and the wave weighs them 64 at a time (a lane sums a
                // block's windows, one atomic). Rounds: usually one (AX_WL = 128, ~100 blocks per pass at config 2
                // with varying qualities); at most 2 blocks of every lane per pass cost 2-5 passes, each with its
                // own sub-batches of 64 (mostly idle lanes) and wave synchronisations.
                uint32_t nzb = 0;
                if (wl_pend) {
#pragma unroll
                    for (uint32_t c = 0; c < AX_CMPW; ++c)
#pragma unroll
                        for (uint32_t b = 0; b < 4u; ++b)
                            nzb |= (((ownc[c] >> (8u * b)) & 0xFFu) != 0u ? 1u : 0u) << (4u * c + b);
                    wlm[lane] = wl_g | (wl_j << 16);
                }
                const uint32_t cnt = (uint32_t)__popc(nzb);  // <= 20
                uint32_t pre = 0, all = 0;
#pragma unroll
                for (uint32_t b = 0; b < 5u; ++b) {
                    const unsigned long long m = __ballot(((cnt >> b) & 1u) != 0u);
                    pre += lanes_below(m) << b;
                    all += (uint32_t)__popcll(m) << b;
                }
                for (uint32_t r0 = 0; r0 < all; r0 += AX_WL) {
                    while (nzb != 0u && pre < r0 + AX_WL) {  // this lane's entries in [r0, r0 + AX_WL)
                        const uint32_t blk = (uint32_t)__builtin_ctz(nzb);
                        nzb &= nzb - 1u;
                        const uint32_t c = blk >> 2;
                        const uint32_t oc = c == 0u ? ownc[0] : (c == 1u ? ownc[1] : (c == 2u ? ownc[2] : (c == 3u ? ownc[3] : ownc[4])));
                        wl[pre - r0] = lane | (blk << 6) | (((oc >> (8u * (blk & 3u))) & 0xFFu) << 11);
                        ++pre;
                    }
                    wave_sync();
                    const uint32_t tot = min(all - r0, AX_WL);
                    for (uint32_t b0 = 0; b0 < tot; b0 += 64u) {
                        // the entry's lane o and the first base of o's piece (a full-wave shuffle, before the branch)
                        const uint32_t en = wl[min(b0 + lane, AX_WL - 1u)];
                        const uint64_t qo = (uint64_t)__shfl((long long)ta, (int)(en & 63u));
                        if (b0 + lane < tot) {
                            const uint32_t o = en & 63u, meta = wlm[o];
                            const uint32_t jb = (meta >> 16) + 8u * ((en >> 6) & 31u);
                            double s = 0.0;
                            if (k >= 8u) {
                                s = weight8(qo + jb, en >> 11);
                            } else {
                                const uint32_t so = (uint32_t)off0s[o];
                                for (uint32_t m = en >> 11; m; m &= m - 1u) {
                                    const uint32_t jj = jb + (uint32_t)__builtin_ctz(m);
                                    s += weight(qo + jj, chg_zero(o, so + jj + 1u, k - 1u));
                                }
                            }
                            add_weight(meta & 0xFFFFu, s);
                        }
                    }
                    wave_sync();
                }
            }
        }
        if (STATS) {
            if (run_phase) c_rn += clock64() - c_s;
            else c_lk += clock64() - c_s;
        }
    }
    const uint64_t c_tot = STATS ? clock64() - c_t0 : 0ull;
    if (has_unit && ad) atomicAdd(&wsum[1], 1ull);  // the wave's last units
    wave_sync();
    const unsigned long long tsum = wsum[0], asum = wsum[1];
    // T and the ambiguous units go out with the workgroup's histogram (LDS_HIST: one atomic instruction per workgroup
    // for all G + 2 counters, after the barrier). One atomic per wave on the counters' cache line, 5,120 of them per
    // launch at config 2 on the same line, cost 35 µs of a 0.22 ms launch (profiles/r05/ab_final_atomics.jsonl).
    if (!LDS_HIST && lane == 0) {
        if (tsum) atomicAdd(&out_a[0], tsum);
        if (asum) atomicAdd(&out_a[1], asum);
    }
    if (STATS) {
        const uint64_t sv[AXS_N] = {s_iter, s_lk, s_rn, s_lkw, s_rnw, s_rwin, s_def, s_fp, s_p2, s_p2v, s_ch, s_seg,
                                    s_qb, s_tal, s_rg, s_spl, s_b4, s_b16, s_b32, s_b64,
                                    lane == 0 ? c_ref : 0ull, lane == 0 ? c_lk : 0ull, lane == 0 ? c_rn : 0ull,
                                    lane == 0 ? c_p2 : 0ull, lane == 0 ? c_tot : 0ull, s_p2n,
                                    lane == 0 ? c_p2f : 0ull, s_p2r, lane == 0 ? c_rpre : 0ull,
                                    lane == 0 ? c_rstg : 0ull, 0ull, lane == 0 ? 1ull : 0ull, 0ull, 0ull, 0ull, 0ull,
                                    0ull};
#pragma unroll
        for (uint32_t i = 0; i < AXS_N; ++i)
            if (sv[i]) atomicAdd(&A.stats[i], (unsigned long long)sv[i]);
        if (lane == 0) {
            atomicMax(&A.stats[AXS_CYC_WAVE_MAX], (unsigned long long)c_tot);
            atomicAdd(&A.stats[AXS_CYC_GEN0 + min(blockIdx.x / 256u, 4u)], (unsigned long long)c_tot);
        }
    }
    if (LDS_HIST) {
        __syncthreads();
        // out_a = {T, ambiguous, U[0 .. G)}: thread 0 and 1 sum the waves' T and ambiguous units, thread 2 + g adds U[g]
        for (uint32_t i = threadIdx.x; i < G + 2u; i += AX_THREADS) {
            unsigned long long x = 0;
            if (i < 2u) {
#pragma unroll
                for (uint32_t w = 0; w < AX_WPB; ++w)
                    x += reinterpret_cast<const unsigned long long*>(
                        smem + hist_bytes + qtab_bytes + w * WAVE_BYTES +
                        (reinterpret_cast<const unsigned char*>(wsum) - wb))[i];
            } else {
                x = hA[i - 2u];
            }
            if (x) atomicAdd(&out_a[i], x);
        }
        for (uint32_t g = threadIdx.x; g < (MODE == KM_LOCAL ? G : 0u); g += AX_THREADS) {
            if (MODE == KM_LOCAL) {
                const double y = hW[g];
                if (y != 0.0) atomicAdd(&out_w[g], y);
            }
        }
    }
}

template <int MODE, bool PAIRED, bool LDS, bool EM, int HW, bool STATS>
void ax_launch_one(const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w, uint32_t n_cus) {
    if (lds > 64 * 1024)  // dynamic LDS above 64 KiB must be allowed (occupancy caps pad it)
        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_ax<MODE, PAIRED, LDS, EM, HW, STATS>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    // persistent waves: at most the blocks that are resident at once (each wave then takes several groups of units
    // and refills its lanes from them)
    static std::mutex mu;
    static size_t cached_lds = 0;
    static int cached_blocks = 0;
    int per_cu = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (cached_lds != lds || cached_blocks == 0) {
            int nb = 0;
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void*>(&k_scan_ax<MODE, PAIRED, LDS, EM, HW, STATS>), AX_THREADS, lds));
            cached_lds = lds;
            cached_blocks = std::max(nb, 1);
        }
        per_cu = cached_blocks;
    }
    grid = std::min<uint32_t>(grid, (uint32_t)per_cu * n_cus);
    hipLaunchKernelGGL((k_scan_ax<MODE, PAIRED, LDS, EM, HW, STATS>), dim3(grid), dim3(AX_THREADS), lds, st, A, src,
                       a, w);
}

// HW by k: 1 (k <= 32), 2 (k <= 64), 3 (k <= 96: the reference's default k = 70), 4 (k <= 128)
template <int MODE, bool PAIRED, bool LDS, bool EM, bool STATS>
void ax_launch_nwc(uint32_t k, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w, uint32_t n_cus) {
    if (k <= 32) ax_launch_one<MODE, PAIRED, LDS, EM, 1, STATS>(A, src, grid, lds, st, a, w, n_cus);
    else if (k <= 64) ax_launch_one<MODE, PAIRED, LDS, EM, 2, STATS>(A, src, grid, lds, st, a, w, n_cus);
    else if (k <= 96) ax_launch_one<MODE, PAIRED, LDS, EM, 3, STATS>(A, src, grid, lds, st, a, w, n_cus);
    else ax_launch_one<MODE, PAIRED, LDS, EM, 4, STATS>(A, src, grid, lds, st, a, w, n_cus);
}

template <int MODE, bool PAIRED>
void ax_launch_mode(bool lds_hist, uint32_t k, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds,
                    hipStream_t st, unsigned long long* a, double* w, uint32_t n_cus) {
    const bool em = src.em_mult != nullptr;
    if (A.stats != nullptr && lds_hist && !em) {
        ax_launch_nwc<MODE, PAIRED, true, false, true>(k, A, src, grid, lds, st, a, w, n_cus);
        return;
    }
    if (lds_hist) {
        if (em) ax_launch_nwc<MODE, PAIRED, true, true, false>(k, A, src, grid, lds, st, a, w, n_cus);
        else ax_launch_nwc<MODE, PAIRED, true, false, false>(k, A, src, grid, lds, st, a, w, n_cus);
    } else {
        if (em) ax_launch_nwc<MODE, PAIRED, false, true, false>(k, A, src, grid, lds, st, a, w, n_cus);
        else ax_launch_nwc<MODE, PAIRED, false, false, false>(k, A, src, grid, lds, st, a, w, n_cus);
    }
}

}  // namespace

namespace speq {

uint32_t ax_effective_load(const speq_device_index* d) { return d->ax_load ? d->ax_load : 35u; }

// Builds the per-k anchor structures of replica d (blocking, on its stream). Returns a table with ok == false when
// k, the group count or the index is outside what the scan supports (a structural limit: `transient` false), or
// the structures would not fit the free HBM at this moment (`transient` true: ensure_ax tries again next time).
//
// The representatives come from the replica's suffix array (k_ax_classify: the median of each k-mer's interval),
// sorted on the GPU by the index build's prefix doubling into a buffer of this build's own and freed with the other
// temporaries: it is read only here (about 52 B per symbol of temporaries while it is sorted, 4 B per symbol while
// the classes are computed). When it does not fit, or the sort fails, the first thread to claim an interval
// represents it (same classes and counts; only the runs per read differ). SPEQ_INJECT_SA_SORT_FAILURE=1 (tests)
// makes the sort fail after its buffer was allocated.
AxTable build_ax(speq_device_index* d, uint32_t k) {
    DeviceGuard g(d->device);
    const auto t0 = std::chrono::steady_clock::now();
    AxTable ax;
    const uint64_t n = d->view.n;
    if (k < 1 || k > AX_MAX_K || n >= (1ull << 30) || d->G > AX_MAX_G) return ax;
    const uint64_t nw64 = (n + 63) / 64 + 4;
    const uint64_t n_gran = (n + 255) / 32 + 2;  // a run from any p < n reads <= AX_NGR granules: padded with END
    const uint64_t gran_bytes = n_gran * 16;
    size_t free_b = 0, total_b = 0;
    HIP_OK(hipMemGetInfo(&free_b, &total_b));
    // gran, codes, owner, text2 + tbad, table + filter (bounds); the EM-only mlo / mhi come later (ensure_ax_em)
    const uint64_t need = gran_bytes + n + (n + 64) * 4 + nw64 * 24 + n * 12;
    if (need > free_b / 10 * 9) {
        ax.transient = true;
        return ax;
    }
    uint32_t* owner = nullptr;
    uint8_t* codes = nullptr;
    uint32_t* sa = nullptr;
    unsigned long long* d_cnt = nullptr;
    std::vector<void*> mine;  // this table's allocations (tracked by the replica once the table is complete)
    auto cleanup = [&] {
        (void)hipStreamSynchronize(d->stream);
        for (void** q : {reinterpret_cast<void**>(&owner), reinterpret_cast<void**>(&codes),
                         reinterpret_cast<void**>(&sa), reinterpret_cast<void**>(&d_cnt)}) {
            if (*q) (void)hipFree(*q);
            *q = nullptr;
        }
    };
    auto alloc = [&](void** pp, uint64_t bytes) {
        HIP_OK(hipMalloc(pp, bytes));
        mine.push_back(*pp);
    };
    try {
        if (!d->d_text2) {  // 2-bit text + non-ACGT bitmap, once per replica
            HIP_OK(hipMalloc(&d->d_text2, nw64 * 16));
            d->track(d->d_text2);
            HIP_OK(hipMalloc(&d->d_tbad, nw64 * 8));
            d->track(d->d_tbad);
            const uint32_t grid = (uint32_t)std::min<uint64_t>((nw64 + 255) / 256, 4096);
            hipLaunchKernelGGL(k_ax_text2, dim3(grid), dim3(256), 0, d->stream, d->d_text, n, d->d_text2, d->d_tbad,
                               nw64);
            HIP_OK(hipGetLastError());
        }
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        if (n * 60 + need < free_b / 10 * 9) {
            HIP_OK(hipMalloc(&sa, n * 4));
            try {
                HIP_OK(hipStreamSynchronize(d->stream));
                const char* inj = std::getenv("SPEQ_INJECT_SA_SORT_FAILURE");
                if (inj && inj[0] == '1') throw DeviceError("build_ax: injected suffix-sort failure");
                gpu_suffix_sort(d->d_text, (uint32_t)n, sa, d->stream, false);
                HIP_OK(hipStreamSynchronize(d->stream));
            } catch (const std::exception&) {
                (void)hipStreamSynchronize(d->stream);
                (void)hipGetLastError();
                (void)hipFree(sa);
                sa = nullptr;  // first claimants represent their k-mers
            }
        }
        alloc(&ax.gran, gran_bytes);
        HIP_OK(hipMalloc(&owner, (n + 1) * 4));
        HIP_OK(hipMalloc(&codes, n + 64));
        HIP_OK(hipMalloc(&d_cnt, 8));
        HIP_OK(hipMemsetAsync(owner, 0xFF, (n + 1) * 4, d->stream));
        HIP_OK(hipMemsetAsync(d_cnt, 0, 8, d->stream));
        const DevView v = search_view(d, k);
        const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 16384);
        hipLaunchKernelGGL(k_ax_classify, dim3(grid), dim3(256), 0, d->stream, v, d->d_text, d->d_tbad, n, k, codes,
                           owner, sa, d_cnt);
        HIP_OK(hipGetLastError());
        const uint32_t pgrid = (uint32_t)std::min<uint64_t>((n_gran + 255) / 256, 16384);
        hipLaunchKernelGGL(k_ax_pack, dim3(pgrid), dim3(256), 0, d->stream, d->d_text2, 2 * nw64, codes, n,
                           reinterpret_cast<u32x4*>(ax.gran), n_gran);
        HIP_OK(hipGetLastError());
        unsigned long long distinct = 0;
        HIP_OK(hipMemcpyAsync(&distinct, d_cnt, 8, hipMemcpyDeviceToHost, d->stream));
        HIP_OK(hipStreamSynchronize(d->stream));
        if (sa) {  // read by k_ax_classify only
            (void)hipFree(sa);
            sa = nullptr;
        }
        ax.distinct = distinct;
        const uint32_t load = ax_effective_load(d);
        ax.nf = std::max<uint64_t>(1, distinct * AX_FILTER_BITS / 64);
        ax.nb = std::max<uint64_t>(1, (uint64_t)((double)distinct * 100.0 / (8.0 * load)) + 1);
        // the m-mer filter (k_ax_mfilter) after the buckets: 16 bits per m-mer, sized by the distinct k-mers plus
        // the m-mers that start no valid k-mer window near a text end (k per text); an undersized filter only
        // passes more m-mers (their windows are deferred as before), it never proves a present window absent
        ax.m = ax_mproof_m(n, k);
        ax.nmf = ax.m ? std::max<uint64_t>(1, (distinct + (uint64_t)d->n_texts * k) * AX_FILTER_BITS / 64) : 0;
        if (ax.m && ax.nb * 64u + ax.nmf * 8u + 16u >= (1ull << 32) - 64) ax.m = 0, ax.nmf = 0;
        if (ax.nb * 64u >= (1ull << 32) - 64 || ax.nf * 8 >= (1ull << 32) - 64) {
            // the scan addresses the tables with 32-bit buffer offsets: leave this k to the other kernels
            cleanup();
            for (void* q : mine) (void)hipFree(q);
            return AxTable{};
        }
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        const uint64_t atab_bytes = ax.nb * 64u + (ax.m ? ax.nmf * 8u + 16u : 0u);
        if (atab_bytes + ax.nf * 8 > free_b / 10 * 9) {  // the table and filters do not fit now: try again later
            cleanup();
            for (void* q : mine) (void)hipFree(q);
            AxTable t;
            t.transient = true;
            return t;
        }
        alloc(&ax.filt, ax.nf * 8);
        HIP_OK(hipMemsetAsync(ax.filt, 0, ax.nf * 8, d->stream));
        alloc(&ax.atab, atab_bytes);
        HIP_OK(hipMemsetAsync(ax.atab, 0xFF, ax.nb * 64u, d->stream));
        if (ax.m) {
            unsigned long long* mf = reinterpret_cast<unsigned long long*>(static_cast<char*>(ax.atab) + ax.nb * 64u);
            HIP_OK(hipMemsetAsync(mf, 0, ax.nmf * 8u + 16u, d->stream));
            hipLaunchKernelGGL(k_ax_mfilter, dim3(grid), dim3(256), 0, d->stream, d->d_text2, d->d_tbad, n, ax.m, mf,
                               ax.nmf);
            HIP_OK(hipGetLastError());
        }
        hipLaunchKernelGGL(k_ax_insert, dim3(grid), dim3(256), 0, d->stream, owner, n, d->d_text2, k, d->d_text_start,
                           d->d_text_group, d->n_texts, reinterpret_cast<unsigned long long*>(ax.atab), ax.nb,
                           reinterpret_cast<unsigned long long*>(ax.filt), ax.nf);
        HIP_OK(hipGetLastError());
        HIP_OK(hipStreamSynchronize(d->stream));
        ax.load = load;
        ax.gran_bytes = gran_bytes;
        ax.bytes = atab_bytes + ax.nf * 8 + gran_bytes;
        ax.ok = true;
    } catch (...) {
        cleanup();
        for (void* q : mine) (void)hipFree(q);
        throw;
    }
    cleanup();
    for (void* q : mine) d->track(q);
    ax.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    startup_trace("per-k structures built");
    return ax;
}

const AxTable* ensure_ax(speq_device_index* d, uint32_t k) {
    if (!d->ax_scan || k < 1 || k > AX_MAX_K) return nullptr;
    std::lock_guard<std::mutex> lk(d->ax_mu);
    auto it = d->axtabs.find(k);
    if (it != d->axtabs.end() && !it->second.ok && it->second.transient) {
        d->axtabs.erase(it);  // it did not fit the free HBM last time: try again
        it = d->axtabs.end();
    }
    if (it == d->axtabs.end()) it = d->axtabs.emplace(k, build_ax(d, k)).first;
    return it->second.ok ? &it->second : nullptr;
}

// The EM-only arrays of table ax (k): allocated and filled on the first EM scan of k (8 B per text position: 1.6 GB
// at config 5, which plain scans never read). Returns false when they do not fit the free HBM.
static bool ensure_ax_em(speq_device_index* d, AxTable* ax, uint32_t k) {
    std::lock_guard<std::mutex> lk(d->ax_mu);
    if (ax->mlo) return true;
    DeviceGuard g(d->device);
    const uint64_t n = d->view.n;
    size_t free_b = 0, total_b = 0;
    HIP_OK(hipMemGetInfo(&free_b, &total_b));
    if ((n + 64) * 8 > free_b / 10 * 9) return false;
    uint32_t* mlo = nullptr;
    uint32_t* mhi = nullptr;
    HIP_OK(hipMalloc(&mlo, (n + 64) * 4));
    if (hipMalloc(&mhi, (n + 64) * 4) != hipSuccess) {
        (void)hipFree(mlo);
        throw DeviceError("ensure_ax_em: hipMalloc failed");
    }
    const DevView v = search_view(d, k);
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_ax_em_intervals, dim3(grid), dim3(256), 0, d->stream, v, d->d_text,
                       reinterpret_cast<const u32x4*>(ax->gran), n, k, mlo, mhi);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(d->stream));
    d->track(mlo);
    d->track(mhi);
    ax->mhi = mhi;
    ax->mlo = mlo;  // last: the unlocked check in launch_ax reads it
    ax->bytes += (n + 64) * 8;
    return true;
}

// Launches k_scan_ax for a read scan (mode 0 global, 1 local) when replica d has (or can build) the structures of
// src.k; returns false when the caller must use another kernel. With src.ax_stats set (speq_scan_reads_device_stats:
// a per-call buffer, so concurrent ordinary scans of the replica never see it), the diagnostic instantiation also adds
// its work counters there.
bool launch_ax(speq_device_index* d, int mode, bool paired, const UnitSrc& src, hipStream_t st, unsigned long long* a,
               double* w) {
    if (src.n_units >= (1ull << 32)) return false;  // 32-bit read indices in the kernel: the other kernels take it
    AxTable* ax = const_cast<AxTable*>(ensure_ax(d, src.k));
    if (!ax) return false;
    if (src.em_mult != nullptr && !ensure_ax_em(d, ax, src.k)) return false;  // EM: the other kernels take it
    AxView A;
    A.gran = reinterpret_cast<const u32x4*>(ax->gran);
    A.mlo = ax->mlo;
    A.mhi = ax->mhi;
    A.atab = reinterpret_cast<const unsigned long long*>(ax->atab);
    A.filt = reinterpret_cast<const unsigned long long*>(ax->filt);
    A.stats = src.ax_stats;
    A.nb = ax->nb;
    A.nf = ax->nf;
    A.n = d->view.n;
    A.gran_bytes = ax->gran_bytes;
    A.m = d->ax_mproof ? ax->m : 0u;
    A.mtiles = d->ax_mproof == 1u ? 1u : 0u;
    A.nmf = A.m ? ax->nmf : 0u;
    A.mf_off = (uint32_t)(ax->nb * 64u);
    A.G = d->G;
    const bool lds_hist = d->G <= LDS_HIST_MAX_G;
    const uint32_t hist_words = lds_hist ? (mode == KM_GLOBAL ? d->G : 2u * d->G) : 0u;
    const size_t lds = ((hist_words * 8u + 15u) & ~15u) + (mode == KM_LOCAL ? QTAB_BYTES : 0u) +
                       (size_t)AX_WPB * (mode == KM_LOCAL ? ax_wave_bytes<KM_LOCAL>() : ax_wave_bytes<KM_GLOBAL>());
    const uint64_t reads = src.n_units;
    uint64_t blocks = (reads + 64 * AX_WPB - 1) / (64 * AX_WPB);
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, d->grid_blocks_ax));
    size_t lds_launch = lds;
    if (d->blocks_per_cu_ax > 0) {
        const size_t pad = (160u * 1024u) / d->blocks_per_cu_ax;
        if (pad > lds_launch) lds_launch = pad & ~(size_t)15;
    }
    const uint32_t grid = (uint32_t)blocks;
    const uint32_t slots = d->n_cus * d->ax_generations;  // (the grid cap: resident blocks per CU x slots)
    if (mode == KM_GLOBAL) {
        if (paired) ax_launch_mode<KM_GLOBAL, true>(lds_hist, src.k, A, src, grid, lds_launch, st, a, w, slots);
        else ax_launch_mode<KM_GLOBAL, false>(lds_hist, src.k, A, src, grid, lds_launch, st, a, w, slots);
    } else {
        if (paired) ax_launch_mode<KM_LOCAL, true>(lds_hist, src.k, A, src, grid, lds_launch, st, a, w, slots);
        else ax_launch_mode<KM_LOCAL, false>(lds_hist, src.k, A, src, grid, lds_launch, st, a, w, slots);
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace speq

namespace speq {
// Loads this translation unit's code object onto the current device (HIP loads a code object at the first use of
// one of its kernels: 30-55 ms for the scan kernels' on the first launch of a `speq scan` run; speq_device_warmup).
void warm_module_ax_scan() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_ax_pack));
}
}  // namespace speq
