// Anchor-and-extend read scan (k_scan_ax) and its per-k structures, for gfx950 (MI355X). DESIGN.md §4e.
//
// Replaces, for every read window, the reference's `search(f_kmers, fm_index, cfg)` + the first-hit tally
// (/root/reference/src/fm_scanner.cpp:153-196 global, :426-471 local, :665-729 paired, :916-962 paired local).
//
// Why: consecutive windows of a read that matches the reference are consecutive positions of the reference text, and
// whether a k-mer is unique to one group is a property of the k-mer, i.e. of ANY of its occurrences. So per k the
// replica keeps the classification of the k-mer that starts at every text position (`cls`, one u32 per position: the
// group, MULTI | SA-interval start, or SENT for a window that crosses a text end or holds an N), plus a hash table
// of one representative position per distinct k-mer (`atab`). A lane takes one READ: it looks its first window up
// once (the anchor: bucket -> fingerprint -> representative p), then compares the read with the 2-bit text at p,
// 32 windows at a time (one XOR per 32 bases), and reads the classes of all matched windows with coalesced 16-B loads
// of cls[p + d]. A mismatch (a SNP against the representative, or a sequencing error) ends the run and the next
// window is looked up again. Every verdict is exact: a window is classified from cls[p'] only after its k bases were
// compared equal with text[p', p' + k), and a window is absent only after the hash chain of its key ran into an empty
// slot without a verified fingerprint match.
//
// Windows whose anchor lookup finds nothing (the k windows over a sequencing error) and windows that matched a text
// position whose class is SENT are DEFERRED: the wave collects them in LDS and resolves them after the per-read
// pass, 64 at a time, one window per lane (phase 2), so one erroneous read does not hold its wave for k lookups.
//
// Cost per read (150 bp, k = 21, no error): one bucket gather + ~4 x (a 3-word text load, eight 16-B class loads,
// one XOR compare, 32 tallies). The k-mer table kernel (k_scan_kt) pays one 64-B bucket gather + a hash + an
// 8-slot compare for EVERY window, and its per-window bookkeeping (cursor, staging, ballots) runs for every lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "device_index.hpp"
#include "scan_device.hpp"
#include "scan_internal.hpp"

namespace {

using namespace speq_dev;

constexpr uint32_t AX_MAX_K = 128;    // longest k the scan takes (AX_CAP - k + 1 windows per segment)
constexpr uint32_t AX_CAP = 192;      // bases of a read a lane stages at once (longer reads: segments of AX_CAP bases)
constexpr uint32_t AX_STREAM = AX_CAP + 16;  // staged bases incl. the 16-B alignment slack before the read
constexpr uint32_t AX_CHUNKS = AX_STREAM / 16;
constexpr uint32_t AX_RUN = 32;       // windows a lane classifies per iteration (one compare, eight 16-B class loads)
constexpr uint32_t AX_PKW = 9;        // staged 2-bit words per lane (AX_STREAM bases + extraction slack)
constexpr uint32_t AX_VWW = 4;        // valid-window words per lane
constexpr uint32_t AX_CGW = 5;        // quality-change words per lane (local mode)
constexpr uint32_t AX_DEF = 512;      // deferred-window entries per wave
constexpr uint32_t AX_VOID = 0xFFFFFFFFu;  // a deferred-list slot reserved by a lane that then kept its windows
constexpr uint32_t AX_SENT = 0xFFFFFFFFu;
constexpr uint32_t AX_MULTI = 0x80000000u;
constexpr uint32_t AX_EMPTY = 0xFFFFFFFFu;
constexpr unsigned long long AX_SLOT_EMPTY = ~0ull;
constexpr uint32_t AX_OOB = 0xFFFFFFF0u;  // buffer offset past every class array (n < 2^30)

static_assert(AX_STREAM % 16 == 0, "chunks of 16 bases");

__host__ __device__ __forceinline__ uint64_t ax_fmix(uint64_t x) {  // murmur3 fmix64 (a bijection)
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

// Hash of a k-mer given as little-endian 2-bit words (base i at bits 2(i % 32) of word i / 32; A C G T = 0 1 2 3);
// words past the k-mer are ignored, so the text side (k_ax_insert) and the read side agree for any NW >= ceil(k/32).
template <int NW>
__device__ __forceinline__ uint64_t ax_hash(const uint64_t (&w)[NW], uint32_t k) {
    uint64_t h = 0x9E3779B97F4A7C15ull * (uint64_t)(k + 1u);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if (32u * (uint32_t)i < k) {
            const uint32_t rem = k - 32u * (uint32_t)i;
            uint64_t x = w[i];
            if (rem < 32u) x &= (1ull << (2u * rem)) - 1ull;
            h = ax_fmix(h ^ x);
        }
    }
    return h;
}
__host__ __device__ __forceinline__ uint32_t ax_bucket(uint64_t h, uint64_t nb) {
    return (uint32_t)(((h >> 32) * nb) >> 32);
}

__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t sh) {  // bits [sh, sh + 64) of hi:lo
    return sh == 0u ? lo : ((lo >> sh) | (hi << (64u - sh)));
}

// bytes of v that are zero -> 0x80 in that byte (exact: no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}
// the 0x80 flags of the four bytes -> bits 0..3
__device__ __forceinline__ uint32_t flags4(uint32_t m) {
    uint32_t y = m >> 7;
    y |= y >> 7;
    y |= y >> 14;
    return y & 0xFu;
}

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
__device__ int ax_search_text(const DevView& I, const Rsrc& R, const uint8_t* __restrict__ t, uint32_t k, uint32_t& lo_out,
                              uint32_t& hi_out) {
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

// Pass A: the class of the k-mer at every text position, and one representative position per distinct k-mer (the
// first to claim owner[lo] of its SA interval). Multi-group k-mers also record their interval end (mhi[lo], for EM).
__global__ void k_ax_classify(DevView I, const uint8_t* __restrict__ text, const uint64_t* __restrict__ tbad,
                              uint64_t n, uint32_t k, uint32_t* __restrict__ cls, uint32_t* __restrict__ mhi,
                              uint32_t* __restrict__ owner, unsigned long long* __restrict__ n_distinct) {
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
        if (!valid) {
            cls[pos] = AX_SENT;
            continue;
        }
        uint32_t lo = 0, hi = 0;
        const int g = ax_search_text(I, R, text + pos, k, lo, hi);
        // g == -1 cannot happen: the window occurs at pos
        cls[pos] = g >= 0 ? (uint32_t)g : (AX_MULTI | lo);
        if (g == -2) mhi[lo] = hi;
        if (atomicCAS(&owner[lo], AX_EMPTY, (uint32_t)pos) == AX_EMPTY) ++claimed;
    }
    if (claimed) atomicAdd(n_distinct, claimed);
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

// Pass B: every representative position inserts {fingerprint, position} into the anchor table (8 slots per 64-B
// bucket, first empty slot in order, linear probing over buckets; no deletions).
__global__ void k_ax_insert(const uint32_t* __restrict__ owner, uint64_t n, const uint64_t* __restrict__ t2, uint32_t k,
                            unsigned long long* __restrict__ atab, uint64_t nb) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = owner[i];
        if (p == AX_EMPTY) continue;
        uint64_t w[4];
        ax_text_words<4>(t2, p, w);
        const uint64_t h = ax_hash<4>(w, k);
        const unsigned long long v = ((unsigned long long)p << 32) | (uint32_t)h;
        uint32_t b = ax_bucket(h, nb);
        for (bool placed = false; !placed; b = (b + 1u == nb) ? 0u : b + 1u)
            for (uint32_t j = 0; j < 8u && !placed; ++j)
                placed = atomicCAS(&atab[(uint64_t)b * 8u + j], AX_SLOT_EMPTY, v) == AX_SLOT_EMPTY;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// The scan
// ---------------------------------------------------------------------------------------------------------------

struct AxView {
    const uint64_t* t2;        // 2-bit text
    const uint32_t* cls;       // class per text position (+ padding)
    const uint32_t* mhi;       // interval end of multi-group k-mers, by interval start (EM)
    const unsigned long long* atab;
    uint64_t nb;               // buckets
    uint64_t n;                // text length
    uint32_t G;
};

// One probe of the anchor table from bucket *b, slot *s: returns the first slot >= *s whose fingerprint matches
// (position in *p), or "absent" when an empty slot comes first; a full bucket without either moves to the next one.
// On a match *b/*s point at that slot (a failed verification resumes at *s + 1).
__device__ __forceinline__ bool ax_probe(const AxView& A, uint32_t fp, uint32_t& b, uint32_t& s, uint32_t& p,
                                         bool active) {
    bool found = false, pending = active;
    while (__ballot(pending) != 0) {
        if (pending) {
            const uint4* pb = reinterpret_cast<const uint4*>(A.atab + (uint64_t)b * 8u);
            const uint4 v0 = pb[0], v1 = pb[1], v2 = pb[2], v3 = pb[3];
            const uint32_t fps[8] = {v0.x, v0.z, v1.x, v1.z, v2.x, v2.z, v3.x, v3.z};
            const uint32_t pos[8] = {v0.y, v0.w, v1.y, v1.w, v2.y, v2.w, v3.y, v3.w};
            uint32_t mm = 0, me = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const bool empty = pos[t] == AX_EMPTY;
                me |= (empty ? 1u : 0u) << t;
                mm |= ((!empty && fps[t] == fp) ? 1u : 0u) << t;
            }
            const uint32_t from = s >= 8u ? 0u : (0xFFu << s) & 0xFFu;
            mm &= from;
            me &= from;
            const uint32_t fm = mm ? (uint32_t)__builtin_ctz(mm) : 8u, fe = me ? (uint32_t)__builtin_ctz(me) : 8u;
            if (fm < fe) {
                s = fm;
                uint32_t pp = pos[0];
#pragma unroll
                for (int t = 1; t < 8; ++t) pp = fm == (uint32_t)t ? pos[t] : pp;
                p = pp;
                found = true;
                pending = false;
            } else if (fe < 8u) {
                pending = false;  // absent
            } else {
                b = (b + 1u == (uint32_t)A.nb) ? 0u : b + 1u;
                s = 0;
            }
        }
    }
    return found;
}

template <int MODE, bool PAIRED, bool LDS_HIST, bool EM, int NWC>
__global__ __launch_bounds__(BLOCK_THREADS) void k_scan_ax(AxView A, UnitSrc src, unsigned long long* __restrict__ out_a,
                                                           double* __restrict__ out_w) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = A.G, k = src.k;
    const uint32_t hist_words = LDS_HIST ? ((MODE == KM_GLOBAL) ? G : 2u * G) : 0u;
    const uint32_t hist_bytes = (hist_words * 8u + 15u) & ~15u;
    unsigned long long* hA = reinterpret_cast<unsigned long long*>(smem);
    double* hW = reinterpret_cast<double*>(hA + G);
    double2* qtab = reinterpret_cast<double2*>(smem + hist_bytes);  // KM_LOCAL
    double* wtab = reinterpret_cast<double*>(qtab + QLUT_LEN);
    const uint32_t qtab_bytes = MODE == KM_LOCAL ? QTAB_BYTES : 0u;
    constexpr uint32_t WAVE_BYTES = 8u * 64u * (AX_PKW + AX_VWW + (MODE == KM_LOCAL ? AX_CGW + 1u : 0u)) +
                                    4u * AX_DEF + 16u + 8u * 64u + 64u;
    unsigned char* wb = smem + hist_bytes + qtab_bytes + wid * WAVE_BYTES;
    uint64_t* pk = reinterpret_cast<uint64_t*>(wb);                 // [AX_PKW][64]
    uint64_t* vwl = pk + AX_PKW * 64u;                               // [AX_VWW][64]
    uint64_t* cg = vwl + AX_VWW * 64u;                               // [AX_CGW][64] (local)
    uint64_t* rbase = cg + (MODE == KM_LOCAL ? AX_CGW * 64u : 0u);   // [64] (local): segment start offsets
    uint32_t* defl = reinterpret_cast<uint32_t*>(rbase + (MODE == KM_LOCAL ? 64u : 0u));  // [AX_DEF]
    uint32_t* defn = defl + AX_DEF;                                  // [4]
    int32_t* ambf = reinterpret_cast<int32_t*>(defn + 4);            // [64] first counted group
    int32_t* ambd = ambf + 64;                                       // [64] another group seen
    uint8_t* off0s = reinterpret_cast<uint8_t*>(ambd + 64);          // [64] alignment slack of each lane's stream

    if (MODE == KM_LOCAL)
        for (uint32_t i = threadIdx.x; i < QLUT_LEN; i += BLOCK_THREADS) {
            const double lut = src.qlut[2 * i], inv = src.qlut[2 * i + 1];
            qtab[i] = make_double2(lut, inv);
            double x = 1.0;  // fm_scanner.cpp:454, k bases of quality i
            for (uint32_t j = 0; j < k; ++j) x = div_rn(x, lut, inv);
            wtab[i] = x;
        }
    if (LDS_HIST)
        for (uint32_t i = threadIdx.x; i < hist_words; i += BLOCK_THREADS) hA[i] = 0ull;
    __syncthreads();
    unsigned long long* gU = out_a + 2;

    // class loads go through a buffer descriptor (dword-aligned 16-B loads; a lane without a run gets an out-of-range
    // offset, which issues no memory request)
    const __amdgpu_buffer_rsrc_t rs_cls =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.cls, (short)0, (int)(uint32_t)((A.n + 256u) * 4u), 0x00020000);
    const uint64_t NWV = (uint64_t)gridDim.x * WAVES_PER_BLOCK;
    const uint64_t gw = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + wid;
    const uint64_t nu = PAIRED ? src.n_units / 2 : src.n_units;
    const uint64_t u0 = nu * gw / NWV, u1 = nu * (gw + 1) / NWV;
    const uint64_t r_begin = PAIRED ? 2 * u0 : u0, r_end = PAIRED ? 2 * u1 : u1;
    const uint32_t segw = AX_CAP - k + 1u;  // windows per segment
    const uint32_t cmpb = k - 1u + AX_RUN;  // bases compared per iteration

    uint32_t t_cnt = 0, amb = 0;

    // run-length tally of the current lane (flushed when the group changes)
    int32_t run_g = -1;
    uint32_t run_n = 0;
    double run_w = 0.0;
    auto flush = [&]() {
        if (run_n) {
            if (LDS_HIST) {
                atomicAdd(&hA[run_g], (unsigned long long)run_n);
                if (MODE == KM_LOCAL) atomicAdd(&hW[run_g], run_w);
            } else {
                atomicAdd(&gU[run_g], (unsigned long long)run_n);
                if (MODE == KM_LOCAL) atomicAdd(&out_w[run_g], run_w);
            }
        }
        run_n = 0;
        run_w = 0.0;
    };

    for (uint64_t r0 = r_begin; r0 < r_end; r0 += 64) {
        const uint64_t r = r0 + lane;
        const bool has = r < r_end;
        const uint64_t rb = has ? src.off[r] : 0, re = has ? src.off[r + 1] : 0;
        const uint64_t L = re - rb;
        const uint64_t W = L >= k ? L - k + 1 : 0;
        const uint32_t nseg = (uint32_t)((W + segw - 1) / segw);
        uint32_t nseg_max = nseg;
        for (uint32_t d = 32; d >= 1; d >>= 1) nseg_max = max(nseg_max, (uint32_t)__shfl_xor((int)nseg_max, (int)d));
        nseg_max = __builtin_amdgcn_readfirstlane(nseg_max);
        int32_t af = -1, ad = 0;  // ambiguity state of this lane's read
        for (uint32_t seg = 0; seg < nseg_max; ++seg) {
            // ---- stage segment `seg`: windows [s, s + wend) of the read, bases [s, s + sb)
            const bool in_seg = seg < nseg;
            const uint64_t s = (uint64_t)seg * segw;
            const uint32_t sb = in_seg ? (uint32_t)(L - s < AX_CAP ? L - s : AX_CAP) : 0u;
            const uint32_t wend = in_seg ? (uint32_t)(W - s < segw ? W - s : segw) : 0u;
            const uint64_t a = rb + s;                       // first base (offset into seq/qual)
            const uint64_t a16 = a & ~15ull;
            const uint32_t off0 = (uint32_t)(a - a16);
            const uint32_t nch = in_seg ? (off0 + sb + 15u) / 16u : 0u;
            uint64_t badw[4] = {~0ull, ~0ull, ~0ull, ~0ull};
            uint64_t cgw[4] = {0ull, 0ull, 0ull, 0ull};
            uint32_t qprev = 0;
            const uint32_t qt = 33u + src.cutoff;  // Phred+33 byte <= qt  <=>  clamp(q, 0, 41) <= cutoff (cutoff < 41)
            const uint32_t qt4 = (qt > 0x7Fu ? 0x7Fu : qt) * 0x01010101u;
#pragma unroll
            for (uint32_t c = 0; c < AX_CHUNKS; ++c) {
                if (c < nch) {
                    const uint4 sv = *reinterpret_cast<const uint4*>(src.seq + a16 + 16u * c);
                    const uint4 qv = *reinterpret_cast<const uint4*>(src.qual + a16 + 16u * c);
                    const uint32_t sd[4] = {sv.x, sv.y, sv.z, sv.w}, qd[4] = {qv.x, qv.y, qv.z, qv.w};
                    uint32_t codes = 0, bad = 0, chg = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint32_t x = sd[i] | 0x20202020u;  // lower case
                        const uint32_t c4 = ((x >> 1) ^ (x >> 2)) & 0x03030303u;  // a c g t/u -> 0 1 2 3
                        codes |= ((c4 | (c4 >> 6) | (c4 >> 12) | (c4 >> 18)) & 0xFFu) << (8 * i);
                        const uint32_t canon = __builtin_amdgcn_perm(0u, 0x74676361u, c4);  // the letter of that code
                        const uint32_t okb = zero_bytes(x ^ canon) | zero_bytes(x ^ 0x75757575u);  // ACGT or U
                        const uint32_t y = qd[i];
                        const uint32_t badq = src.cutoff >= 41u
                                                  ? 0x80808080u
                                                  : (((0x80808080u | qt4) - (y & 0x7F7F7F7Fu)) & ~y & 0x80808080u);
                        bad |= flags4((~okb & 0x80808080u) | badq) << (4 * i);
                        if (MODE == KM_LOCAL) {
                            const uint32_t prev = (y << 8) | (qprev >> 24);
                            chg |= flags4(~zero_bytes(y ^ prev) & 0x80808080u) << (4 * i);
                            qprev = y;
                        }
                    }
                    reinterpret_cast<uint32_t*>(pk + (c >> 1) * 64u + lane)[c & 1u] = codes;
                    badw[c >> 2] &= ~(0xFFFFull << (16u * (c & 3u)));
                    badw[c >> 2] |= (uint64_t)bad << (16u * (c & 3u));
                    if (MODE == KM_LOCAL) cgw[c >> 2] |= (uint64_t)chg << (16u * (c & 3u));
                }
            }
            // valid windows: AND of k consecutive "good" bits (doubling), then shifted to the read's first base
            uint64_t ok[4] = {~badw[0], ~badw[1], ~badw[2], ~badw[3]};
            for (uint32_t len = 1; len < k;) {
                const uint32_t sft = min(len, k - len);
                const uint32_t ws = sft >> 6, bs = sft & 63u;
                uint64_t nx[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint64_t lo = (i + ws < 4) ? ok[i + ws] : 0ull;
                    const uint64_t hi = (i + ws + 1 < 4) ? ok[i + ws + 1] : 0ull;
                    nx[i] = ok[i] & funnel(lo, hi, bs);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) ok[i] = nx[i];
                len += sft;
            }
            uint64_t vw[AX_VWW];
#pragma unroll
            for (uint32_t i = 0; i < AX_VWW; ++i) {
                const uint64_t lo = i < 4 ? ok[i] : 0ull, hi = i + 1 < 4 ? ok[i + 1] : 0ull;
                uint64_t v = funnel(lo, hi, off0);
                const uint32_t bit0 = 64u * i;
                if (wend <= bit0) v = 0;
                else if (wend < bit0 + 64u) v &= (1ull << (wend - bit0)) - 1ull;
                vw[i] = v;
                vwl[i * 64u + lane] = v;
                t_cnt += (uint32_t)__popcll(v);
            }
            if (MODE == KM_LOCAL) {
#pragma unroll
                for (uint32_t i = 0; i < AX_CGW; ++i) cg[i * 64u + lane] = i < 4 ? cgw[i] : 0ull;
                rbase[lane] = a;
            }
            off0s[lane] = (uint8_t)off0;
            if (lane == 0) defn[0] = 0;
            wave_sync();

            // per-lane readers of the staged stream
            auto read_words = [&](uint32_t o, uint32_t base, uint64_t(&w)[NWC]) {  // NWC words at stream base `base`
                const uint32_t idx = base >> 5, sh = 2u * (base & 31u);
                uint64_t raw[NWC + 1];
#pragma unroll
                for (int i = 0; i <= NWC; ++i) raw[i] = (idx + i < AX_PKW) ? pk[(idx + i) * 64u + o] : 0ull;
#pragma unroll
                for (int i = 0; i < NWC; ++i) w[i] = funnel(raw[i], raw[i + 1], sh);
            };
            auto next_valid = [&](uint32_t j) -> uint32_t {  // first valid window >= j (or wend)
                uint32_t res = wend;
#pragma unroll
                for (int i = (int)AX_VWW - 1; i >= 0; --i) {
                    const uint32_t b0 = 64u * (uint32_t)i;
                    uint64_t v = vw[i];
                    if (j > b0) v = (j - b0 >= 64u) ? 0ull : (v & (~0ull << (j - b0)));
                    if (v) res = b0 + (uint32_t)__builtin_ctzll(v);
                }
                return res;
            };
            auto defer_push = [&](uint32_t o, uint32_t jj) -> bool {
                const uint32_t slot = atomicAdd(&defn[0], 1u);
                if (slot < AX_DEF) defl[slot] = o | (jj << 6);
                return slot < AX_DEF;
            };
            // Phred weight of window jj (bases a + jj ..) of the read whose segment starts at `base` (global offset)
            auto weight = [&](const uint8_t* qbase, bool uniform, uint32_t qcur) -> double {
                if (uniform) return wtab[qcur];
                double x = 1.0;
                for (uint32_t i = 0; i < k; ++i) {
                    int q = (int)qbase[i] - 33;
                    q = q < 0 ? 0 : (q > 41 ? 41 : q);
                    const double2 t = qtab[q];
                    x = div_rn(x, t.x, t.y);  // == x / t.x (fm_scanner.cpp:454)
                }
                return x;
            };
            auto uniform_at = [&](uint32_t o, uint32_t off0o, uint32_t jj) -> bool {  // no quality change in (jj, jj + k)
                // stream bits [off0o + jj + 1, off0o + jj + k): k - 1 <= 127 bits over <= 3 words
                uint32_t b = off0o + jj + 1u, left = k - 1u;
                bool u = true;
                while (left) {
                    const uint32_t w = b >> 6, sh = b & 63u, span = min(64u - sh, left);
                    const uint64_t m = span == 64u ? ~0ull : ((1ull << span) - 1ull);
                    u = u && ((cg[w * 64u + o] >> sh) & m) == 0;
                    b += span;
                    left -= span;
                }
                return u;
            };

            // ---- phase 1: one read per lane
            uint32_t j = 0;
            bool lookup = true;        // the next window needs an anchor lookup
            uint64_t p = 0;            // text position of window j when !lookup
            int32_t last_mm = -1;      // base (relative to the segment) of the last observed mismatch
            uint32_t rb_b = 0, rb_s = 0;  // probe resume after a failed verification
            bool resume = false;
            int32_t qpos = -1;         // local mode: window whose (uniform) quality is qcur
            uint32_t qcur = 0;
            for (;;) {
                if (lookup && j < wend) j = next_valid(j);
                const bool act = j < wend;
                if (__ballot(act) == 0) break;
                uint64_t ra[NWC];
                read_words(lane, off0 + j, ra);
                // anchor lookup
                uint32_t pp = 0;
                const bool need = act && lookup;
                const uint64_t h = ax_hash<NWC>(ra, k);
                if (need && !resume) {
                    rb_b = ax_bucket(h, A.nb);
                    rb_s = 0;
                }
                if (need) resume = false;
                const bool cand = ax_probe(A, (uint32_t)h, rb_b, rb_s, pp, need);
                const bool have = act && (!lookup || cand);
                const uint64_t pt = lookup ? (uint64_t)pp : p;
                // text words and the classes of up to AX_RUN windows at pt (both depend only on pt)
                uint64_t tw[NWC];
                uint32_t cv[AX_RUN];
                {
                    const uint64_t ps = have ? pt : 0;
                    ax_text_words<NWC>(A.t2, ps, tw);
                    const uint32_t boff = have ? (uint32_t)(ps * 4u) : AX_OOB;
#pragma unroll
                    for (uint32_t c = 0; c < AX_RUN / 4; ++c) {
                        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_cls, boff + 16u * c, 0, 0);
                        cv[4 * c] = v[0];
                        cv[4 * c + 1] = v[1];
                        cv[4 * c + 2] = v[2];
                        cv[4 * c + 3] = v[3];
                    }
                }
                // compare read [j, j + cmpb) with text [pt, pt + cmpb): e = bases equal before the first mismatch
                uint32_t e = cmpb;
#pragma unroll
                for (int i = NWC - 1; i >= 0; --i) {
                    uint64_t x = ra[i] ^ tw[i];
                    const uint32_t b0 = 32u * (uint32_t)i;
                    if (cmpb <= b0) x = 0;
                    else if (cmpb < b0 + 32u) x &= (1ull << (2u * (cmpb - b0))) - 1ull;
                    if (x) e = b0 + ((uint32_t)__builtin_ctzll(x) >> 1);
                }
                bool absent = act && lookup && !cand;
                bool fpfail = false;
                if (have && lookup && e < k) {  // fingerprint collision: resume probing after that slot
                    fpfail = true;
                    resume = true;
                    ++rb_s;
                }
                const bool run = have && !fpfail;
                uint32_t R = 0;
                if (run) {
                    R = e >= k - 1u ? e - (k - 1u) : 0u;
                    R = min(R, AX_RUN);
                    R = min(R, wend - j);
                }
                // ---- absent anchor: defer the windows that share the mismatch (or the next k - 1), skip past them
                if (absent) {
                    uint32_t dend = (last_mm >= (int32_t)j && last_mm < (int32_t)(j + k)) ? (uint32_t)last_mm : j + k - 1u;
                    dend = min(dend, wend - 1u);
                    uint32_t cnt = 0;
                    for (uint32_t w = j + 1; w <= dend; ++w) cnt += (uint32_t)((vwl[(w >> 6) * 64u + lane] >> (w & 63u)) & 1u);
                    bool ok_def = true;
                    if (cnt) {
                        const uint32_t slot0 = atomicAdd(&defn[0], cnt);
                        ok_def = slot0 + cnt <= AX_DEF;
                        if (ok_def) {
                            uint32_t sl = slot0;
                            for (uint32_t w = j + 1; w <= dend; ++w)
                                if ((vwl[(w >> 6) * 64u + lane] >> (w & 63u)) & 1u) defl[sl++] = lane | (w << 6);
                        } else {  // no room: the windows stay in this pass; void the slots reserved below the end
                            for (uint32_t sl = slot0; sl < AX_DEF && sl < slot0 + cnt; ++sl) defl[sl] = AX_VOID;
                        }
                    }
                    j = ok_def ? dend + 1u : j + 1u;
                    lookup = true;
                    last_mm = -1;
                }
                // ---- tally the run: windows j .. j + R - 1 at text positions pt .. pt + R - 1
                uint32_t vwin = 0;
                if (run) {
                    const uint32_t w0 = j >> 6, sh = j & 63u;
                    uint64_t lo = 0, hi = 0;
#pragma unroll
                    for (uint32_t i = 0; i < AX_VWW; ++i) {
                        lo = w0 == i ? vw[i] : lo;
                        hi = w0 + 1u == i ? vw[i] : hi;
                    }
                    vwin = (uint32_t)funnel(lo, hi, sh);
                }
                bool stop = false;
                uint32_t rstop = R;
#pragma unroll
                for (uint32_t c = 0; c < AX_RUN / 4; ++c) {
                    if (__ballot(run && 4u * c < R) == 0) break;
#pragma unroll
                    for (uint32_t t = 0; t < 4; ++t) {
                        const uint32_t d = 4u * c + t;
                        const uint32_t cl = cv[d];
                        bool v = run && !stop && d < R && ((vwin >> d) & 1u);
                        if (v && cl == AX_SENT) {  // matched bases, but no valid text window there: look it up later
                            v = false;
                            if (!defer_push(lane, j + d)) {
                                stop = true;
                                rstop = d;
                            }
                        }
                        if (v && cl < G) {
                            double wgt = 0.0;
                            if (MODE == KM_LOCAL) {
                                const uint32_t jj = j + d;
                                const bool uni = uniform_at(lane, off0, jj);
                                if (uni && !(qpos >= 0 && jj - (uint32_t)qpos < k)) {
                                    int q = (int)src.qual[a + jj] - 33;
                                    qcur = (uint32_t)(q < 0 ? 0 : (q > 41 ? 41 : q));
                                    qpos = (int32_t)jj;
                                } else if (uni) {
                                    qpos = (int32_t)jj;
                                }
                                wgt = weight(src.qual + a + jj, uni, qcur);
                            }
                            if ((int32_t)cl != run_g) {
                                flush();
                                run_g = (int32_t)cl;
                            }
                            ++run_n;
                            if (MODE == KM_LOCAL) run_w += wgt;
                            if (af < 0) af = (int32_t)cl;
                            else if ((int32_t)cl != af) ad = 1;
                        } else if (EM && v && (cl & AX_MULTI)) {
                            const uint32_t lo = cl & ~AX_MULTI;
                            atomicAdd(&src.em_mult[lo], 1u);
                            src.em_hi[lo] = A.mhi[lo];
                        }
                    }
                }
                if (run) {
                    if (stop) {
                        j += rstop;
                        lookup = true;
                        last_mm = -1;
                    } else {
                        const bool mism = e < cmpb;  // the run ended at a mismatch (base j + e)
                        if (mism && R < wend - j) last_mm = (int32_t)(j + e);
                        j += R;
                        if (mism || R == 0) {
                            lookup = true;
                        } else {
                            lookup = false;
                            p = pt + R;
                        }
                        if (R == 0) lookup = true;
                    }
                }
            }
            flush();

            // ---- phase 2: the deferred windows of the wave, one per lane
            ambf[lane] = af;
            ambd[lane] = ad;
            wave_sync();
            const uint32_t n2 = min(__builtin_amdgcn_readfirstlane(defn[0]), AX_DEF);
            for (uint32_t base = 0; base < n2; base += 64) {
                const uint32_t idx = base + lane;
                const bool act = idx < n2;
                uint32_t ent = act ? defl[idx] : AX_VOID;
                const bool act2 = ent != AX_VOID;
                if (!act2) ent = 0u;
                const uint32_t o = ent & 63u, jj = ent >> 6;
                const uint32_t off0o = off0s[o];
                uint64_t ra[NWC];
                read_words(o, off0o + jj, ra);
                const uint64_t h = ax_hash<NWC>(ra, k);
                uint32_t b = act2 ? ax_bucket(h, A.nb) : 0u, sl = 0, pp = 0;
                bool pend = act2, found = false;
                uint32_t cl = AX_SENT;
                while (__ballot(pend) != 0) {
                    const bool c = ax_probe(A, (uint32_t)h, b, sl, pp, pend);
                    uint64_t tw[NWC];
                    ax_text_words<NWC>(A.t2, (pend && c) ? pp : 0u, tw);
                    const u32x4 cvv = __builtin_amdgcn_raw_buffer_load_b128(rs_cls, (pend && c) ? pp * 4u : AX_OOB,
                                                                             0, 0);
                    if (pend) {
                        if (!c) {
                            pend = false;  // absent
                        } else {
                            bool eq = true;
#pragma unroll
                            for (int i = 0; i < NWC; ++i) {
                                uint64_t x = ra[i] ^ tw[i];
                                const uint32_t b0 = 32u * (uint32_t)i;
                                if (k <= b0) x = 0;
                                else if (k < b0 + 32u) x &= (1ull << (2u * (k - b0))) - 1ull;
                                eq = eq && x == 0;
                            }
                            if (eq) {
                                found = true;
                                cl = cvv[0];
                                pend = false;
                            } else {
                                ++sl;  // fingerprint collision: keep probing
                            }
                        }
                    }
                }
                if (found && cl < G) {
                    double wgt = 0.0;
                    if (MODE == KM_LOCAL) {
                        const uint8_t* qb = src.qual + rbase[o] + jj;
                        const bool uni = uniform_at(o, off0o, jj);
                        int q = (int)qb[0] - 33;
                        q = q < 0 ? 0 : (q > 41 ? 41 : q);
                        wgt = weight(qb, uni, (uint32_t)q);
                    }
                    if (LDS_HIST) {
                        atomicAdd(&hA[cl], 1ull);
                        if (MODE == KM_LOCAL) atomicAdd(&hW[cl], wgt);
                    } else {
                        atomicAdd(&gU[cl], 1ull);
                        if (MODE == KM_LOCAL) atomicAdd(&out_w[cl], wgt);
                    }
                    const int32_t old = atomicCAS(&ambf[o], -1, (int32_t)cl);
                    if (old != -1 && old != (int32_t)cl) ambd[o] = 1;
                } else if (EM && found && (cl & AX_MULTI) && cl != AX_SENT) {
                    const uint32_t lo = cl & ~AX_MULTI;
                    atomicAdd(&src.em_mult[lo], 1u);
                    src.em_hi[lo] = A.mhi[lo];
                }
            }
            wave_sync();
            af = ambf[lane];
            ad = ambd[lane];
            wave_sync();
        }
        // ---- ambiguity of the unit (read, or mate pair in lanes 2i, 2i + 1)
        if (PAIRED) {
            const int32_t of = __shfl_xor(af, 1), od = __shfl_xor(ad, 1);
            const bool amb_pair = ad || od || (af >= 0 && of >= 0 && af != of);
            if (has && (lane & 1u) == 0u && amb_pair) ++amb;
        } else if (has && ad) {
            ++amb;
        }
    }

    const unsigned long long tsum = wave_sum<unsigned long long>((unsigned long long)t_cnt);
    const unsigned long long asum = wave_sum<unsigned long long>((unsigned long long)amb);
    if (lane == 0) {
        if (tsum) atomicAdd(&out_a[0], tsum);
        if (asum) atomicAdd(&out_a[1], asum);
    }
    if (LDS_HIST) {
        __syncthreads();
        for (uint32_t g = threadIdx.x; g < G; g += BLOCK_THREADS) {
            const unsigned long long x = hA[g];
            if (x) atomicAdd(&gU[g], x);
            if (MODE == KM_LOCAL) {
                const double y = hW[g];
                if (y != 0.0) atomicAdd(&out_w[g], y);
            }
        }
    }
}

template <int MODE>
constexpr uint32_t ax_wave_bytes() {
    return 8u * 64u * (AX_PKW + AX_VWW + (MODE == KM_LOCAL ? AX_CGW + 1u : 0u)) + 4u * AX_DEF + 16u + 8u * 64u + 64u;
}

template <int MODE, bool PAIRED, bool LDS, bool EM, int NWC>
void ax_launch_one(const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w) {
    if (lds > 64 * 1024)  // dynamic LDS above 64 KiB must be allowed (occupancy caps pad it)
        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_ax<MODE, PAIRED, LDS, EM, NWC>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL((k_scan_ax<MODE, PAIRED, LDS, EM, NWC>), dim3(grid), dim3(BLOCK_THREADS), lds, st, A, src, a, w);
}

template <int MODE, bool PAIRED, bool LDS, bool EM>
void ax_launch_nwc(uint32_t nwc, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w) {
    switch (nwc) {
        case 2: ax_launch_one<MODE, PAIRED, LDS, EM, 2>(A, src, grid, lds, st, a, w); break;
        case 3: ax_launch_one<MODE, PAIRED, LDS, EM, 3>(A, src, grid, lds, st, a, w); break;
        case 4: ax_launch_one<MODE, PAIRED, LDS, EM, 4>(A, src, grid, lds, st, a, w); break;
        default: ax_launch_one<MODE, PAIRED, LDS, EM, 5>(A, src, grid, lds, st, a, w); break;
    }
}

template <int MODE, bool PAIRED, bool LDS>
void ax_launch_em(uint32_t nwc, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                  unsigned long long* a, double* w) {
    if (src.em_mult != nullptr) ax_launch_nwc<MODE, PAIRED, LDS, true>(nwc, A, src, grid, lds, st, a, w);
    else ax_launch_nwc<MODE, PAIRED, LDS, false>(nwc, A, src, grid, lds, st, a, w);
}

}  // namespace

namespace speq {

// Builds the per-k anchor structures of replica d (blocking, on its stream). Returns a table with ok == false when
// k or the index is outside what the scan supports, or the structures would not fit the free HBM.
AxTable build_ax(speq_device_index* d, uint32_t k) {
    DeviceGuard g(d->device);
    const auto t0 = std::chrono::steady_clock::now();
    AxTable ax;
    const uint64_t n = d->view.n;
    if (k < 1 || k > AX_MAX_K || n >= (1ull << 30)) return ax;
    const uint64_t nw64 = (n + 63) / 64 + 4;
    size_t free_b = 0, total_b = 0;
    HIP_OK(hipMemGetInfo(&free_b, &total_b));
    const uint64_t need = (n + 256) * 4 * 3 + nw64 * 24 + n * 8;  // cls, mhi, owner, text2 + tbad, table (bound)
    if (need > free_b / 10 * 9) return ax;
    uint32_t* owner = nullptr;
    unsigned long long* d_cnt = nullptr;
    auto cleanup = [&] {
        (void)hipStreamSynchronize(d->stream);
        if (owner) (void)hipFree(owner);
        if (d_cnt) (void)hipFree(d_cnt);
        owner = nullptr;
        d_cnt = nullptr;
    };
    try {
        if (!d->d_text2) {  // 2-bit text + non-ACGT bitmap, once per replica
            HIP_OK(hipMalloc(&d->d_text2, nw64 * 16));
            HIP_OK(hipMalloc(&d->d_tbad, nw64 * 8));
            d->track(d->d_text2);
            d->track(d->d_tbad);
            const uint32_t grid = (uint32_t)std::min<uint64_t>((nw64 + 255) / 256, 4096);
            hipLaunchKernelGGL(k_ax_text2, dim3(grid), dim3(256), 0, d->stream, d->d_text, n, d->d_text2, d->d_tbad,
                               nw64);
            HIP_OK(hipGetLastError());
        }
        HIP_OK(hipMalloc(&ax.cls, (n + 256) * 4));
        d->track(ax.cls);
        HIP_OK(hipMalloc(&ax.mhi, (n + 1) * 4));
        d->track(ax.mhi);
        HIP_OK(hipMalloc(&owner, (n + 1) * 4));
        HIP_OK(hipMalloc(&d_cnt, 8));
        HIP_OK(hipMemsetAsync(ax.cls, 0xFF, (n + 256) * 4, d->stream));
        HIP_OK(hipMemsetAsync(owner, 0xFF, (n + 1) * 4, d->stream));
        HIP_OK(hipMemsetAsync(d_cnt, 0, 8, d->stream));
        const DevView v = search_view(d, k);
        const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 16384);
        hipLaunchKernelGGL(k_ax_classify, dim3(grid), dim3(256), 0, d->stream, v, d->d_text, d->d_tbad, n, k, ax.cls,
                           ax.mhi, owner, d_cnt);
        HIP_OK(hipGetLastError());
        unsigned long long distinct = 0;
        HIP_OK(hipMemcpyAsync(&distinct, d_cnt, 8, hipMemcpyDeviceToHost, d->stream));
        HIP_OK(hipStreamSynchronize(d->stream));
        ax.distinct = distinct;
        ax.nb = std::max<uint64_t>(1, (uint64_t)((double)distinct * 100.0 / (8.0 * d->ax_load)) + 1);
        if (ax.nb >= (1ull << 32)) throw DeviceError("anchor table too large");
        HIP_OK(hipMalloc(&ax.atab, ax.nb * 64));
        d->track(ax.atab);
        HIP_OK(hipMemsetAsync(ax.atab, 0xFF, ax.nb * 64, d->stream));
        hipLaunchKernelGGL(k_ax_insert, dim3(grid), dim3(256), 0, d->stream, owner, n, d->d_text2, k,
                           reinterpret_cast<unsigned long long*>(ax.atab), ax.nb);
        HIP_OK(hipGetLastError());
        HIP_OK(hipStreamSynchronize(d->stream));
        ax.bytes = ax.nb * 64 + (n + 256) * 4 + (n + 1) * 4;
        ax.ok = true;
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
    ax.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return ax;
}

const AxTable* ensure_ax(speq_device_index* d, uint32_t k) {
    if (!d->ax_scan || k < 1 || k > AX_MAX_K) return nullptr;
    std::lock_guard<std::mutex> lk(d->ax_mu);
    auto it = d->axtabs.find(k);
    if (it == d->axtabs.end()) it = d->axtabs.emplace(k, build_ax(d, k)).first;
    return it->second.ok ? &it->second : nullptr;
}

// Launches k_scan_ax for a read scan (mode 0 global, 1 local) when replica d has (or can build) the structures of
// src.k; returns false when the caller must use another kernel.
bool launch_ax(speq_device_index* d, int mode, bool paired, const UnitSrc& src, hipStream_t st, unsigned long long* a,
               double* w) {
    const AxTable* ax = ensure_ax(d, src.k);
    if (!ax) return false;
    AxView A;
    A.t2 = d->d_text2;
    A.cls = ax->cls;
    A.mhi = ax->mhi;
    A.atab = reinterpret_cast<const unsigned long long*>(ax->atab);
    A.nb = ax->nb;
    A.n = d->view.n;
    A.G = d->G;
    const bool lds_hist = d->G <= LDS_HIST_MAX_G;
    const uint32_t hist_words = lds_hist ? (mode == KM_GLOBAL ? d->G : 2u * d->G) : 0u;
    const size_t lds = ((hist_words * 8u + 15u) & ~15u) + (mode == KM_LOCAL ? QTAB_BYTES : 0u) +
                       (size_t)WAVES_PER_BLOCK * (mode == KM_LOCAL ? ax_wave_bytes<KM_LOCAL>() : ax_wave_bytes<KM_GLOBAL>());
    const uint64_t reads = src.n_units;
    uint64_t blocks = (reads + 64 * WAVES_PER_BLOCK - 1) / (64 * WAVES_PER_BLOCK);
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, d->grid_blocks_ax));
    size_t lds_launch = lds;
    if (d->blocks_per_cu_ax > 0) {
        const size_t pad = (160u * 1024u) / d->blocks_per_cu_ax;
        if (pad > lds_launch) lds_launch = pad & ~(size_t)15;
    }
    const uint32_t nwc = (src.k + 31u + 31u) / 32u;  // words covering k - 1 + AX_RUN bases
    const uint32_t grid = (uint32_t)blocks;
#define SPEQ_AX(M, P)                                                                        \
    do {                                                                                     \
        if (lds_hist) ax_launch_em<M, P, true>(nwc, A, src, grid, lds_launch, st, a, w);     \
        else ax_launch_em<M, P, false>(nwc, A, src, grid, lds_launch, st, a, w);             \
    } while (0)
    if (mode == KM_GLOBAL) {
        if (paired) SPEQ_AX(KM_GLOBAL, true);
        else SPEQ_AX(KM_GLOBAL, false);
    } else {
        if (paired) SPEQ_AX(KM_LOCAL, true);
        else SPEQ_AX(KM_LOCAL, false);
    }
#undef SPEQ_AX
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace speq
