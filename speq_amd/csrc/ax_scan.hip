// Anchor-and-extend read scan (k_scan_ax) and its per-k structures, for gfx950 (MI355X). DESIGN.md §4e.
//
// Replaces, for every read window, the reference's `search(f_kmers, fm_index, cfg)` + the first-hit tally
// (/root/reference/src/fm_scanner.cpp:153-196 global, :426-471 local, :665-729 paired, :916-962 paired local).
//
// Why: consecutive windows of a read that matches the reference are consecutive positions of the reference text, and
// whether a k-mer is unique to one group is a property of the k-mer, i.e. of ANY of its occurrences. So per k the
// replica keeps the class of the k-mer that starts at every text position (`cls`, 1 byte per position when the
// index has <= 253 groups, else 2: the group, MULTI, or SENT for a window that crosses a text end or holds an N), plus
// a hash table of one representative position per distinct k-mer (`atab`). A lane takes one READ: it looks one window
// up (the anchor: bucket -> fingerprint -> representative p), then compares the read with the 2-bit text at p, 64
// windows at a time (one XOR per 32 bases), and reads the classes of the matched windows (64 bytes: four 16-B loads).
// A mismatch (a SNP against the representative, or a sequencing error) ends the run and the next window is looked up
// again. Every verdict is exact: a window is classified from cls[p'] only after its k bases were compared equal with
// text[p', p' + k), and a window is absent only after its key's chain in the anchor table ran into an empty slot
// without a verified fingerprint match (or its bits are missing from the table's blocked Bloom filter, which holds
// every k-mer of the texts).
//
// Windows whose anchor lookup finds nothing (the k windows over a sequencing error) and windows that matched a text
// position whose class is SENT are DEFERRED: the wave collects them in LDS and, after the per-read pass, tests them
// against the Bloom filter (four per lane per round trip) and looks the survivors up one per lane, so one erroneous
// read does not hold its wave for k lookups.
//
// What bounds it (profiles/r02): the per-CU vector-memory path, which serves the lanes' scattered 16-B loads one
// cache line per lane; so the classes are bytes (a 64-window run is four loads, not sixteen), a load group is issued
// only when some lane of the wave needs it, and one iteration costs one round trip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <type_traits>
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
constexpr uint32_t AX_RUN = 64;       // windows a lane classifies per iteration (one compare, 64 class bytes)
constexpr uint32_t AX_VWW = 4;        // valid-window words per lane
constexpr uint32_t AX_SCH = 64 * AX_CHUNKS;     // 16-base chunks of a wave's staged stream (every lane's segment)
constexpr uint32_t AX_CSW = AX_SCH / 2 + 8;     // 2-bit code words (u64) of the stream, + read-past slack
constexpr uint32_t AX_BSW = AX_SCH / 2 + 16;    // 1-bit-per-base words (u32) of the stream (bad / quality change)
constexpr uint32_t AX_DEF = 1024;     // deferred-window entries per wave (u16: lane | window << 6)
constexpr uint32_t AX_F = 4;          // deferred windows a lane tests against the filter per round trip
constexpr uint32_t AX_EMPTY = 0xFFFFFFFFu;
constexpr uint16_t AX_VOID = 0xFFFFu;  // a deferred-list slot reserved by a lane that then kept its windows
constexpr unsigned long long AX_SLOT_EMPTY = ~0ull;
constexpr uint32_t AX_OOB = 0xFFFFFFF0u;  // buffer offset past every array (n < 2^30)
constexpr uint32_t AX_FILTER_BITS = 16;   // Bloom filter bits per distinct k-mer (3 bits set per k-mer, one 64-bit word)
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

static_assert(AX_STREAM % 16 == 0, "chunks of 16 bases");
static_assert(AX_CAP < 1024, "deferred entries hold the window in 10 bits");

// class values (CW bytes per text position): groups 0 .. G-1 < NONE; NONE is never stored
template <int CW>
struct AxCls {
    static constexpr uint32_t SENT = CW == 1 ? 0xFFu : 0xFFFFu;
    static constexpr uint32_t MULTI = SENT - 1u;
    static constexpr uint32_t NONE = SENT - 2u;
    static constexpr uint32_t MAX_G = NONE;
    static constexpr uint32_t PER = 4 / CW;                                   // classes per dword
    static constexpr uint32_t REP = CW == 1 ? 0x01010101u : 0x00010001u;      // broadcast factor
    static constexpr uint32_t FLAGS = CW == 1 ? 0x80808080u : 0x80008000u;    // top bit of every element
    static constexpr uint32_t LOW7 = CW == 1 ? 0x7F7F7F7Fu : 0x7FFF7FFFu;
};

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
// Bloom filter of the distinct k-mers: one 64-bit word per key, three bits in it
__host__ __device__ __forceinline__ uint32_t ax_fword(uint64_t h, uint64_t nf) {
    return (uint32_t)((((h >> 24) & 0xFFFFFFFFull) * nf) >> 32);
}
__host__ __device__ __forceinline__ uint64_t ax_fbits(uint64_t h) {
    return (1ull << (h & 63u)) | (1ull << ((h >> 6) & 63u)) | (1ull << ((h >> 12) & 63u));
}

__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t sh) {  // bits [sh, sh + 64) of hi:lo
    return sh == 0u ? lo : ((lo >> sh) | (hi << (64u - sh)));
}

// bytes of v that are zero -> 0x80 in that byte (exact: no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}
// the same per element of a class dword
template <int CW>
__device__ __forceinline__ uint32_t zero_elems(uint32_t v) {
    return ~(((v & AxCls<CW>::LOW7) + AxCls<CW>::LOW7) | v) & AxCls<CW>::FLAGS;
}
// the 0x80 flags of the four bytes -> bits 0..3
__device__ __forceinline__ uint32_t flags4(uint32_t m) {
    uint32_t y = m >> 7;
    y |= y >> 7;
    y |= y >> 14;
    return y & 0xFu;
}
// bits 0 .. PER-1 of b -> the top bit of each element of a class dword
template <int CW>
__device__ __forceinline__ uint32_t spread(uint32_t b) {
    if (CW == 1) return ((b * 0x00204081u) & 0x01010101u) << 7;
    return ((b * 0x00008001u) & 0x00010001u) << 15;
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

// Pass A: the class of the k-mer at every text position, and one representative position per distinct k-mer (the
// first to claim owner[lo] of its SA interval). Multi-group k-mers also record their interval: mlo[pos] = its start
// and mhi[start] = its end (EM histograms).
template <int CW>
__global__ void k_ax_classify(DevView I, const uint8_t* __restrict__ text, const uint64_t* __restrict__ tbad,
                              uint64_t n, uint32_t k, void* __restrict__ cls_v, uint32_t* __restrict__ mlo,
                              uint32_t* __restrict__ mhi, uint32_t* __restrict__ owner,
                              unsigned long long* __restrict__ n_distinct) {
    using T = typename std::conditional<CW == 1, uint8_t, uint16_t>::type;
    T* cls = static_cast<T*>(cls_v);
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
            cls[pos] = (T)AxCls<CW>::SENT;
            continue;
        }
        uint32_t lo = 0, hi = 0;
        const int g = ax_search_text(I, R, text + pos, k, lo, hi);
        // g == -1 cannot happen: the window occurs at pos
        cls[pos] = (T)(g >= 0 ? (uint32_t)g : AxCls<CW>::MULTI);
        if (g == -2) {
            mlo[pos] = lo;
            mhi[lo] = hi;
        }
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
// bucket, first empty slot in order, linear probing over buckets; no deletions) and sets its filter bits.
__global__ void k_ax_insert(const uint32_t* __restrict__ owner, uint64_t n, const uint64_t* __restrict__ t2, uint32_t k,
                            unsigned long long* __restrict__ atab, uint64_t nb, unsigned long long* __restrict__ filt,
                            uint64_t nf) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = owner[i];
        if (p == AX_EMPTY) continue;
        uint64_t w[4];
        ax_text_words<4>(t2, p, w);
        const uint64_t h = ax_hash<4>(w, k);
        atomicOr(&filt[ax_fword(h, nf)], (unsigned long long)ax_fbits(h));
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
    const void* cls;           // class per text position (CW bytes each, + padding)
    const uint32_t* mlo;       // SA interval start of the multi-group k-mer at a text position (EM)
    const uint32_t* mhi;       // its end, by interval start (EM)
    const unsigned long long* atab;
    const unsigned long long* filt;
    uint64_t nb;               // buckets
    uint64_t nf;               // filter words
    uint64_t n;                // text length
    uint64_t t2_bytes;         // bytes of the 2-bit text (incl. padding)
    uint64_t cls_bytes;        // bytes of cls (incl. padding)
    uint32_t G;
};

// One probe of the anchor table from bucket *b, slot *s: the first slot >= *s whose fingerprint matches (position in
// *p), or "absent" when an empty slot comes first; a full bucket without either moves to the next one. On a match
// *s is that slot (a failed verification resumes at *s + 1). Phase 2 only (phase 1 resolves its buckets inline).
__device__ __forceinline__ bool ax_probe(const AxView& A, const __amdgpu_buffer_rsrc_t& rs_atab, uint32_t fp,
                                         uint32_t& b, uint32_t& s, uint32_t& p, bool active) {
    bool found = false, pending = active;
    while (__ballot(pending) != 0) {
        const uint32_t boff = pending ? b * 64u : AX_OOB;
        const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff, 0, 0);
        const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 16u, 0, 0);
        const u32x4 v2 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 32u, 0, 0);
        const u32x4 v3 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 48u, 0, 0);
        if (pending) {
            const uint32_t fps[8] = {v0[0], v0[2], v1[0], v1[2], v2[0], v2[2], v3[0], v3[2]};
            const uint32_t pos[8] = {v0[1], v0[3], v1[1], v1[3], v2[1], v2[3], v3[1], v3[3]};
            uint32_t mm = 0, me = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const bool empty = pos[t] == AX_EMPTY;
                me |= (empty ? 1u : 0u) << t;
                mm |= ((!empty && fps[t] == fp) ? 1u : 0u) << t;
            }
            const uint32_t from = s >= 8u ? 0u : ((0xFFu << s) & 0xFFu);
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

template <int MODE>
constexpr uint32_t ax_wave_bytes() {
    // codes | vw | (local: quality-change stream, rbase) | deferred list (u16; the bad-base stream before phase 1) |
    // counters | ambiguity | stream base per lane (u16)
    static_assert(2u * AX_DEF >= 4u * AX_BSW, "the bad-base stream lives in the deferred list");
    return 8u * AX_CSW + 8u * 64u * AX_VWW + (MODE == KM_LOCAL ? 4u * AX_BSW + 8u * 64u : 0u) + 2u * AX_DEF + 16u +
           8u * 64u + 128u;
}

#ifndef SPEQ_AX_PROBE  // timing probes (scripts/ax_probe.py A/B only; results are wrong): 1 staging only, 2 no phase 2,
                       // 3 nothing but the read offsets, 4 no counter flush at the end,
                       // 5 staging alone without its global loads, 6 staging alone without the counter flush
#define SPEQ_AX_PROBE 0
#endif
#ifndef SPEQ_AX_WPB  // waves per workgroup of k_scan_ax (A/B knob)
#define SPEQ_AX_WPB 4
#endif
constexpr uint32_t AX_WPB = SPEQ_AX_WPB, AX_THREADS = 64 * SPEQ_AX_WPB;
#ifndef SPEQ_AX_SU  // staging: stream instructions per load batch (A/B knob)
#define SPEQ_AX_SU 4
#endif
#ifndef SPEQ_AX_MIN_WAVES  // minimum waves per SIMD the register allocator must allow, k <= 33 (A/B knob)
#define SPEQ_AX_MIN_WAVES 4
#endif
#ifndef SPEQ_AX_MIN_WAVES4  // the same for 34 <= k <= 65 (four compare words)
#define SPEQ_AX_MIN_WAVES4 4
#endif
#ifndef SPEQ_AX_MIN_WAVES6  // and 66 <= k <= 128 (six words): 3 waves, 168 VGPRs without most spills, win 12 % at
#define SPEQ_AX_MIN_WAVES6 3  // k = 70 and lose 17 % at k = 21 (profiles/r02/ax_variants_probes.jsonl)
#endif
// local (Phred-weighted) mode holds more live state than global mode: at 4 waves it spilled 54-60 registers per lane
// (k <= 65); 3 waves (168 VGPRs, 36 / 8 spills) win 5 % at k = 21, 3 % at k = 31 and 28 % at k = 45 (0.1 % errors;
// 9-34 % at 0.5 %), 2 waves lose (profiles/r02/ax_variants_local_waves.jsonl)
#ifndef SPEQ_AX_MIN_WAVES_LOCAL  // local mode, k <= 33
#define SPEQ_AX_MIN_WAVES_LOCAL 3
#endif
#ifndef SPEQ_AX_MIN_WAVES4_LOCAL  // local mode, 34 <= k <= 65
#define SPEQ_AX_MIN_WAVES4_LOCAL 3
#endif
#ifndef SPEQ_AX_MIN_WAVES6_LOCAL  // local mode, 66 <= k <= 128 (2 waves, no spills, lose 17-29 %:
                                   // profiles/r02/ax_variants_local_k70_waves.jsonl)
#define SPEQ_AX_MIN_WAVES6_LOCAL SPEQ_AX_MIN_WAVES6
#endif
#ifndef SPEQ_AX_MIN_WAVES_CW2  // two-byte classes (> 253 groups; 0 = as for one-byte classes): their run loop holds
#define SPEQ_AX_MIN_WAVES_CW2 3   // twice the class registers and spilled 91-104 per lane at 4 waves; 3 waves win 30-33 %
#endif                            // at k = 21 / 31 global, 300 groups (profiles/r02/ax_variants_cw2_waves.jsonl)
template <int MODE, int NWC, int CW>
constexpr int ax_min_waves() {
    return (CW == 2 && SPEQ_AX_MIN_WAVES_CW2 > 0) ? SPEQ_AX_MIN_WAVES_CW2 : NWC >= 6 ? (MODE == KM_LOCAL ? SPEQ_AX_MIN_WAVES6_LOCAL : SPEQ_AX_MIN_WAVES6)
                    : (NWC >= 4 ? (MODE == KM_LOCAL ? SPEQ_AX_MIN_WAVES4_LOCAL : SPEQ_AX_MIN_WAVES4)
                                : (MODE == KM_LOCAL ? SPEQ_AX_MIN_WAVES_LOCAL : SPEQ_AX_MIN_WAVES));
}
template <int MODE, bool PAIRED, bool LDS_HIST, bool EM, int NWC, int CW>
__global__ __launch_bounds__(AX_THREADS, (ax_min_waves<MODE, NWC, CW>())) void k_scan_ax(AxView A, UnitSrc src, unsigned long long* __restrict__ out_a,
                                                           double* __restrict__ out_w) {
    using C = AxCls<CW>;
    constexpr uint32_t PER = C::PER;
    constexpr uint32_t RUNW = AX_RUN / PER;  // class dwords of one run
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
    constexpr uint32_t WAVE_BYTES = ax_wave_bytes<MODE>();
    unsigned char* wb = smem + hist_bytes + qtab_bytes + wid * WAVE_BYTES;
    uint64_t* cs = reinterpret_cast<uint64_t*>(wb);                 // [AX_CSW] 2-bit codes of the wave's stream
    uint64_t* vwl = cs + AX_CSW;                                     // [AX_VWW][64] valid windows per lane
    uint32_t* cgs = reinterpret_cast<uint32_t*>(vwl + AX_VWW * 64u); // [AX_BSW] quality-change bits (local)
    uint64_t* rbase = reinterpret_cast<uint64_t*>(cgs + (MODE == KM_LOCAL ? AX_BSW : 0u));  // [64] (local)
    uint16_t* defl = reinterpret_cast<uint16_t*>(rbase + (MODE == KM_LOCAL ? 64u : 0u));  // [AX_DEF]
    uint32_t* bss = reinterpret_cast<uint32_t*>(defl);               // [AX_BSW] bad-base bits (staging only)
    uint32_t* defn = reinterpret_cast<uint32_t*>(defl + AX_DEF);     // [4]: entries, survivors
    int32_t* ambf = reinterpret_cast<int32_t*>(defn + 4);            // [64] first counted group
    int32_t* ambd = ambf + 64;                                       // [64] another group seen
    uint16_t* sbs = reinterpret_cast<uint16_t*>(ambd + 64);          // [64] stream base of each lane's segment

    if (MODE == KM_LOCAL)
        for (uint32_t i = threadIdx.x; i < QLUT_LEN; i += AX_THREADS) {
            const double lut = src.qlut[2 * i], inv = src.qlut[2 * i + 1];
            qtab[i] = make_double2(lut, inv);
            double x = 1.0;  // fm_scanner.cpp:454, k bases of quality i
            for (uint32_t j = 0; j < k; ++j) x = div_rn(x, lut, inv);
            wtab[i] = x;
        }
    if (LDS_HIST)
        for (uint32_t i = threadIdx.x; i < hist_words; i += AX_THREADS) hA[i] = 0ull;
    __syncthreads();
    unsigned long long* gU = out_a + 2;

    // every table is read through a buffer descriptor: 16-B loads need only dword alignment, and a lane that has
    // nothing to load gets an out-of-range offset, which issues no memory request
    const __amdgpu_buffer_rsrc_t rs_cls =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.cls, (short)0, (int)(uint32_t)A.cls_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_atab =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.atab, (short)0, (int)(uint32_t)(A.nb * 64u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_t2 =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.t2, (short)0, (int)(uint32_t)A.t2_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_filt =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.filt, (short)0, (int)(uint32_t)(A.nf * 8u), 0x00020000);
    const uint64_t NWV = (uint64_t)gridDim.x * AX_WPB;
    const uint64_t gw = (uint64_t)blockIdx.x * AX_WPB + wid;
    const uint64_t nu = PAIRED ? src.n_units / 2 : src.n_units;
    // groups of 64 reads (32 mate pairs), dealt to the waves round robin: the waves in flight sweep the read buffers
    // front to back together (a wave owning one contiguous range ran the staging loads at a third of the HBM rate)
    const uint64_t r_end = PAIRED ? 2 * nu : nu;
    const uint64_t n_groups = (r_end + 63) / 64;
    const uint32_t segw = AX_CAP - k + 1u;  // windows per segment
    const uint32_t cmpb = k - 1u + AX_RUN;  // bases compared per iteration

    uint32_t t_cnt = 0, amb = 0;

    auto add_count = [&](uint32_t g, uint32_t cnt, double wsum) {
        if (LDS_HIST) {
            atomicAdd(&hA[g], (unsigned long long)cnt);
            if (MODE == KM_LOCAL) atomicAdd(&hW[g], wsum);
        } else {
            atomicAdd(&gU[g], (unsigned long long)cnt);
            if (MODE == KM_LOCAL) atomicAdd(&out_w[g], wsum);
        }
    };
    // one class from a text position (phase 2)
    auto load_class = [&](uint32_t p, bool act) -> uint32_t {
        const uint32_t by = p * (uint32_t)CW;
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rs_cls, act ? (by & ~3u) : AX_OOB, 0, 0);
        return (v >> (8u * (by & 3u))) & C::SENT;
    };

    for (uint64_t grp = gw; grp < n_groups; grp += NWV) {
        const uint64_t r0 = grp * 64;
        const uint64_t r = r0 + lane;
        const bool has = r < r_end;
        const uint64_t rb = has ? src.off[r] : 0, re = has ? src.off[r + 1] : 0;
        const uint64_t L = re - rb;
        const uint64_t W = L >= k ? L - k + 1 : 0;
        const uint32_t nseg = (uint32_t)((W + segw - 1) / segw);
        // the wave's largest segment count, bit by bit from the top (ballots: no shuffle address registers, which
        // the compiler hoists out of the loops and spills)
        uint32_t nseg_max = 0;
        if (__ballot(nseg > 1u) == 0) {
            nseg_max = __ballot(nseg != 0u) != 0 ? 1u : 0u;
        } else {
            for (int b = 31; b >= 0; --b) {  // greedy: set bit b when some lane reaches the candidate
                const uint32_t cand = nseg_max | (1u << b);
                if (__ballot(nseg >= cand) != 0) nseg_max = cand;
            }
        }
        int32_t af = -1, ad = 0;  // ambiguity state of this lane's read
        for (uint32_t seg = 0; seg < nseg_max; ++seg) {
#if SPEQ_AX_PROBE == 3  // timing probe only (wrong results): read offsets, no staging
            if (nseg_max > 0u) continue;
#endif
            // ---- stage segment `seg` (windows [s, s + wend) of each lane's read, bases [s, s + sb)) as ONE stream
            // of 16-base chunks: lane o's chunks are [pre_o, pre_o + nch_o), so its base b sits at stream position
            // 16 pre_o + b (b counted from the chunk-aligned a16). The wave decodes the stream 64 chunks per
            // instruction, each lane a whole chunk found by a binary search over the lanes' chunk offsets: the 16-B
            // loads of one instruction cover a few consecutive reads (coalesced) instead of 64 reads 150 B apart.
            const bool in_seg = seg < nseg;
            const uint64_t s = (uint64_t)seg * segw;
            const uint32_t sb = in_seg ? (uint32_t)(L - s < AX_CAP ? L - s : AX_CAP) : 0u;
            const uint32_t wend = in_seg ? (uint32_t)(W - s < segw ? W - s : segw) : 0u;
            const uint64_t a = rb + s;                       // first base (offset into seq/qual)
            const uint64_t a16 = a & ~15ull;
            const uint32_t off0 = (uint32_t)(a - a16);
            const uint32_t nch = in_seg ? (off0 + sb + 15u) / 16u : 0u;
            // exclusive prefix sum of the chunk counts (< 16) by bit planes: per bit, a ballot and a count of the lanes
            // below this one (mbcnt)
            static_assert(AX_CHUNKS < 16, "chunk counts in four bits");
            uint32_t pre = 0, nch_tot = 0;
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const unsigned long long bb = __ballot((nch >> b) & 1u);
                pre += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
                nch_tot += (uint32_t)__popcll(bb) << b;
            }
            const uint32_t sbase = 16u * pre + off0;        // stream position of the segment's first base
            const uint64_t gofs = a16 - 16ull * pre;        // byte offset of stream chunk c in this lane's frame: + 16 c
            const uint32_t qt = 33u + src.cutoff;  // Phred+33 byte <= qt  <=>  clamp(q, 0, 41) <= cutoff (cutoff < 41)
            const uint32_t qt4 = (qt > 0x7Fu ? 0x7Fu : qt) * 0x01010101u;
            const uint32_t allbad = src.cutoff >= 41u ? 0x80808080u : 0u;  // every window fails the quality filter
            uint32_t qcarry = 0;  // local: last quality dword of the previous instruction's lane 63
            constexpr uint32_t SU = SPEQ_AX_SU;  // stream instructions whose loads are in flight together
            for (uint32_t c0 = 0; c0 < nch_tot; c0 += 64u * SU) {
                uint4 sv[SU], qv[SU];
#pragma unroll
                for (uint32_t u = 0; u < SU; ++u) {
                    const uint32_t c = min(c0 + 64u * u + lane, nch_tot - 1u);
                    uint32_t o = 0;  // the lane whose segment holds chunk c: the last o with pre_o <= c
#pragma unroll
                    for (uint32_t d = 32; d >= 1; d >>= 1)
                        o = ((uint32_t)__shfl((int)pre, (int)(o + d)) <= c) ? o + d : o;
                    const uint64_t go = (uint64_t)__shfl((long long)gofs, (int)o) + 16ull * c;
#if SPEQ_AX_PROBE == 5  // timing probe only (wrong results): staging without the global loads
                    sv[u] = make_uint4((uint32_t)go, (uint32_t)go * 3u, (uint32_t)go * 5u, (uint32_t)go * 7u);
                    qv[u] = make_uint4(0x49494949u ^ (uint32_t)go, 0x49494949u, 0x49494949u, 0x49494949u);
#else
                    sv[u] = *reinterpret_cast<const uint4*>(src.seq + go);
                    qv[u] = *reinterpret_cast<const uint4*>(src.qual + go);
#endif
                }
#pragma unroll
                for (uint32_t u = 0; u < SU; ++u) {
                    const uint32_t c = c0 + 64u * u + lane;
                    const uint32_t sd[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
                    const uint32_t qd[4] = {qv[u].x, qv[u].y, qv[u].z, qv[u].w};
                    uint32_t qprev = 0;
                    if (MODE == KM_LOCAL) {  // the byte before the chunk: the previous chunk's last quality
                        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)qv[u].w, 0x138, 0xF, 0xF, false);
                        qprev = lane == 0 ? qcarry : up;
                        qcarry = __builtin_amdgcn_readlane(qv[u].w, 63);
                    }
                    uint32_t codes = 0, bad = 0, chg = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint32_t x = sd[i] | 0x20202020u;  // lower case
                        const uint32_t c4 = ((x >> 1) ^ (x >> 2)) & 0x03030303u;  // a c g t/u -> 0 1 2 3
                        codes |= ((c4 | (c4 >> 6) | (c4 >> 12) | (c4 >> 18)) & 0xFFu) << (8 * i);
                        const uint32_t canon = __builtin_amdgcn_perm(0u, 0x74676361u, c4);  // the letter of that code
                        const uint32_t okb = zero_bytes(x ^ canon) | zero_bytes(x ^ 0x75757575u);  // ACGT or U
                        const uint32_t y = qd[i];
                        const uint32_t badq = (((0x80808080u | qt4) - (y & 0x7F7F7F7Fu)) & ~y & 0x80808080u) | allbad;
                        bad |= flags4((~okb & 0x80808080u) | badq) << (4 * i);
                        if (MODE == KM_LOCAL) {
                            const uint32_t prev = (y << 8) | (qprev >> 24);
                            chg |= flags4(~zero_bytes(y ^ prev) & 0x80808080u) << (4 * i);
                            qprev = y;
                        }
                    }
                    if (c < nch_tot) {
                        reinterpret_cast<uint32_t*>(cs)[c] = codes;
                        reinterpret_cast<uint16_t*>(bss)[c] = (uint16_t)bad;
                        if (MODE == KM_LOCAL) reinterpret_cast<uint16_t*>(cgs)[c] = (uint16_t)chg;
                    }
                }
            }
            wave_sync();
            // this lane's bad-base bits (256 from a16; chunks past its segment are bad)
            uint64_t badw[4];
            {
                const uint32_t d0 = pre >> 1, sh = 16u * (pre & 1u);
                uint32_t bw[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) bw[i] = bss[min(d0 + (uint32_t)i, AX_BSW - 1u)];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint64_t lo = (uint64_t)bw[2 * i] | ((uint64_t)bw[2 * i + 1] << 32);
                    const uint64_t hi = (uint64_t)bw[2 * i + 2];
                    uint64_t v = sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
                    const uint32_t b0 = 64u * (uint32_t)i, nb = 16u * nch;  // bits of this lane's chunks
                    if (nb <= b0) v = ~0ull;
                    else if (nb < b0 + 64u) v |= ~0ull << (nb - b0);
                    badw[i] = v;
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
                    uint64_t lo = 0ull, hi = 0ull;  // ok[i + ws], ok[i + ws + 1] (zero past the end), no indexing
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        lo = (uint32_t)(t - i) == ws ? ok[t] : lo;
                        hi = (uint32_t)(t - i) == ws + 1u ? ok[t] : hi;
                    }
                    nx[i] = ok[i] & funnel(lo, hi, bs);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) ok[i] = nx[i];
                len += sft;
            }
#pragma unroll
            for (uint32_t i = 0; i < AX_VWW; ++i) {
                const uint64_t lo = i < 4 ? ok[i] : 0ull, hi = i + 1 < 4 ? ok[i + 1] : 0ull;
                uint64_t v = funnel(lo, hi, off0);
                const uint32_t bit0 = 64u * i;
                if (wend <= bit0) v = 0;
                else if (wend < bit0 + 64u) v &= (1ull << (wend - bit0)) - 1ull;
                vwl[i * 64u + lane] = v;
                t_cnt += (uint32_t)__popcll(v);
            }
            if (MODE == KM_LOCAL) rbase[lane] = a;
            sbs[lane] = (uint16_t)sbase;
            wave_sync();  // the bad-base stream (in the deferred list) is read by every lane before the list is reset
            if (lane == 0) {
                defn[0] = 0;
                defn[1] = 0;
            }
            wave_sync();

            // per-lane readers of the staged stream
            auto read_words = [&](uint32_t base, uint64_t(&w)[NWC]) {  // NWC code words at stream position `base`
                const uint32_t idx = base >> 5, sh = 2u * (base & 31u);
                uint64_t raw[NWC + 1];
#pragma unroll
                for (int i = 0; i <= NWC; ++i) raw[i] = cs[min(idx + (uint32_t)i, AX_CSW - 1u)];
#pragma unroll
                for (int i = 0; i < NWC; ++i) w[i] = funnel(raw[i], raw[i + 1], sh);
            };
            auto vbits = [&](uint32_t b) -> uint64_t {  // this lane's valid-window bits b .. b + 63 (0 past the end)
                const uint32_t w0 = b >> 6, s6 = b & 63u;
                const uint64_t lo = w0 < AX_VWW ? vwl[w0 * 64u + lane] : 0ull;
                const uint64_t hi = w0 + 1u < AX_VWW ? vwl[(w0 + 1u) * 64u + lane] : 0ull;
                return funnel(lo, hi, s6);
            };
            auto next_valid = [&](uint32_t j) -> uint32_t {  // first valid window >= j (or wend)
                uint32_t res = wend;
#pragma unroll
                for (int i = (int)AX_VWW - 1; i >= 0; --i) {
                    const uint32_t b0 = 64u * (uint32_t)i;
                    uint64_t v = vwl[(uint32_t)i * 64u + lane];
                    if (j > b0) v = (j - b0 >= 64u) ? 0ull : (v & (~0ull << (j - b0)));
                    if (v) res = b0 + (uint32_t)__builtin_ctzll(v);
                }
                return res;
            };
            auto defer_push = [&](uint32_t o, uint32_t jj) -> bool {
                const uint32_t slot = atomicAdd(&defn[0], 1u);
                if (slot < AX_DEF) defl[slot] = (uint16_t)(o | (jj << 6));
                return slot < AX_DEF;
            };
            // Phred weight of a window whose first quality byte is at qbase (fm_scanner.cpp:454)
            auto weight = [&](const uint8_t* qbase, bool uniform, uint32_t qcur) -> double {
                if (uniform) return wtab[qcur];
                double x = 1.0;
                for (uint32_t i = 0; i < k; ++i) {
                    int q = (int)qbase[i] - 33;
                    q = q < 0 ? 0 : (q > 41 ? 41 : q);
                    const double2 t = qtab[q];
                    x = div_rn(x, t.x, t.y);  // == x / t.x
                }
                return x;
            };
            // quality-change bits of the stream over positions [x, x + len) all zero (local mode)
            auto chg_zero = [&](uint32_t x, uint32_t len) -> bool {
                uint32_t left = len;
                bool u = true;
                while (left) {
                    const uint32_t w = x >> 5, sh = x & 31u, span = min(32u - sh, left);
                    const uint32_t mk = span == 32u ? ~0u : ((1u << span) - 1u);
                    u = u && (w >= AX_BSW || ((cgs[w] >> sh) & mk) == 0);
                    x += span;
                    left -= span;
                }
                return u;
            };

#if SPEQ_AX_PROBE == 1 || SPEQ_AX_PROBE == 5 || SPEQ_AX_PROBE == 6  // timing probe only (wrong results): staging alone
            if (wend > 0u) continue;
#endif
            // ---- phase 1: one read per lane, one memory round trip per iteration: a lane either probes the anchor
            // table (its candidate is compared in the next iteration) or extends a run by up to AX_RUN windows
            uint32_t j = 0;
            uint32_t st = wend > 0 ? 0u : 2u;  // 0: look window j up, 1: extend from text position p, 2: done
            bool verify = false;       // st 1: p came from the anchor table (window j itself not compared yet)
            uint64_t p = 0;
            int32_t last_mm = -1;      // base (relative to the segment) of the last observed mismatch
            uint32_t pb = 0, ps = 0;   // probe position of the current lookup (bucket, first slot)
            bool resume = false;       // continue the current lookup at (pb, ps): full bucket, or failed verification
            uint32_t gcur = C::NONE;   // the group of this read's last counted run (the fast path's guess)
            for (;;) {
                if (st == 0u) {
                    j = next_valid(j);
                    if (j >= wend) st = 2u;
                }
                if (__ballot(st != 2u) == 0) break;
                const bool lk = st == 0u, rn = st == 1u;
                uint64_t ra[NWC];
                read_words(sbase + j, ra);
                const uint64_t h = ax_hash<NWC>(ra, k);
                if (lk && !resume) {
                    pb = ax_bucket(h, A.nb);
                    ps = 0;
                }
                // ---- this iteration's loads: a bucket (lookup lanes), text words + classes (run lanes), the quality
                // of window j (local mode); a group is issued only when some lane of the wave needs it
                u32x4 q0 = {0u, 0u, 0u, 0u}, q1 = q0, q2 = q0, q3 = q0;
                if (__ballot(lk) != 0) {
                    const uint32_t boff = lk ? pb * 64u : AX_OOB;
                    q0 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff, 0, 0);
                    q1 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 16u, 0, 0);
                    q2 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 32u, 0, 0);
                    q3 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 48u, 0, 0);
                }
                uint64_t traw[NWC + 1];
                uint32_t craw[RUNW + 1];
                uint32_t qj = 0;
                const bool any_rn = __ballot(rn) != 0;
                if (any_rn) {
                    const uint32_t toff = rn ? (uint32_t)((p >> 5) * 8u) : AX_OOB;
#pragma unroll
                    for (int i = 0; i <= NWC; ++i) {
                        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_t2, toff + 8u * (uint32_t)i, 0, 0);
                        traw[i] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
                    }
                    const uint32_t cby = (uint32_t)(p * (uint32_t)CW);
                    const uint32_t coff = rn ? (cby & ~3u) : AX_OOB;
#pragma unroll
                    for (uint32_t c = 0; c < RUNW / 4; ++c) {
                        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_cls, coff + 16u * c, 0, 0);
                        craw[4 * c] = v[0];
                        craw[4 * c + 1] = v[1];
                        craw[4 * c + 2] = v[2];
                        craw[4 * c + 3] = v[3];
                    }
                    craw[RUNW] = __builtin_amdgcn_raw_buffer_load_b32(rs_cls, coff + 4u * RUNW, 0, 0);
                    if (MODE == KM_LOCAL) qj = src.qual[a + (rn ? j : 0u)];
                }

                // ---- lookup lanes: resolve the bucket
                if (lk) {
                    const uint32_t fps[8] = {q0[0], q0[2], q1[0], q1[2], q2[0], q2[2], q3[0], q3[2]};
                    const uint32_t pos[8] = {q0[1], q0[3], q1[1], q1[3], q2[1], q2[3], q3[1], q3[3]};
                    uint32_t mm = 0, me = 0;
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const bool empty = pos[t] == AX_EMPTY;
                        me |= (empty ? 1u : 0u) << t;
                        mm |= ((!empty && fps[t] == (uint32_t)h) ? 1u : 0u) << t;
                    }
                    const uint32_t from = ps >= 8u ? 0u : ((0xFFu << ps) & 0xFFu);
                    mm &= from;
                    me &= from;
                    const uint32_t fm = mm ? (uint32_t)__builtin_ctz(mm) : 8u, fe = me ? (uint32_t)__builtin_ctz(me) : 8u;
                    if (fm < fe) {  // candidate: compared with the text in the next iteration
                        uint32_t pp = pos[0];
#pragma unroll
                        for (int t = 1; t < 8; ++t) pp = fm == (uint32_t)t ? pos[t] : pp;
                        p = pp;
                        ps = fm;
                        st = 1u;
                        verify = true;
                        resume = false;
                    } else if (fe < 8u) {
                        // absent: defer the windows that share the mismatch (or the next k - 1), skip past them
                        resume = false;
                        uint32_t dend = (last_mm >= (int32_t)j && last_mm < (int32_t)(j + k)) ? (uint32_t)last_mm
                                                                                               : j + k - 1u;
                        dend = min(dend, wend - 1u);
                        // the valid windows of (j, dend] as two 64-bit masks (dend - j <= k - 1 <= 127)
                        const uint32_t span = dend - j;
                        uint64_t dm0 = vbits(j + 1u), dm1 = span > 64u ? vbits(j + 65u) : 0ull;
                        dm0 &= span >= 64u ? ~0ull : ((1ull << span) - 1ull);
                        if (span > 64u) dm1 &= span - 64u >= 64u ? ~0ull : ((1ull << (span - 64u)) - 1ull);
                        const uint32_t cnt = (uint32_t)__popcll(dm0) + (uint32_t)__popcll(dm1);
                        bool ok_def = true;
                        if (cnt) {
                            const uint32_t slot0 = atomicAdd(&defn[0], cnt);
                            ok_def = slot0 + cnt <= AX_DEF;
                            if (ok_def) {
                                uint32_t sl = slot0;
                                for (uint64_t t = dm0; t; t &= t - 1)
                                    defl[sl++] = (uint16_t)(lane | ((j + 1u + (uint32_t)__builtin_ctzll(t)) << 6));
                                for (uint64_t t = dm1; t; t &= t - 1)
                                    defl[sl++] = (uint16_t)(lane | ((j + 65u + (uint32_t)__builtin_ctzll(t)) << 6));
                            } else {  // no room: the windows stay with this lane; void the slots reserved below the end
                                for (uint32_t sl = slot0; sl < AX_DEF && sl < slot0 + cnt; ++sl) defl[sl] = AX_VOID;
                            }
                        }
                        j = ok_def ? dend + 1u : j + 1u;
                        last_mm = -1;
                    } else {  // full bucket without the key or an empty slot: the next bucket
                        pb = pb + 1u == (uint32_t)A.nb ? 0u : pb + 1u;
                        ps = 0;
                        resume = true;
                    }
                }

                // ---- run lanes: compare read [j, j + cmpb) with text [p, p + cmpb), classify the matched windows
                if (any_rn && rn) {
                    const uint32_t sh = 2u * (uint32_t)(p & 31u);
                    uint32_t e = cmpb;
#pragma unroll
                    for (int i = NWC - 1; i >= 0; --i) {
                        uint64_t x = ra[i] ^ funnel(traw[i], traw[i + 1], sh);
                        const uint32_t b0 = 32u * (uint32_t)i;
                        if (cmpb <= b0) x = 0;
                        else if (cmpb < b0 + 32u) x &= (1ull << (2u * (cmpb - b0))) - 1ull;
                        if (x) e = b0 + ((uint32_t)__builtin_ctzll(x) >> 1);
                    }
                    if (verify && e < k) {  // fingerprint collision: resume probing after that slot
                        st = 0u;
                        resume = true;
                        ++ps;
                    } else {
                        uint32_t R = e - (k - 1u);  // e >= k - 1: a candidate matched k bases, a run k - 1
                        R = min(R, AX_RUN);
                        R = min(R, wend - j);
                        uint64_t m;
                        {
                            const uint32_t w0 = j >> 6, s6 = j & 63u;
                            const uint64_t lo = vwl[w0 * 64u + lane];
                            const uint64_t hi = w0 + 1u < AX_VWW ? vwl[(w0 + 1u) * 64u + lane] : 0ull;
                            m = funnel(lo, hi, s6) & (R >= 64u ? ~0ull : ((1ull << R) - 1ull));
                        }
                        // the run's classes, aligned so that window d is element d
                        const uint32_t ca = (uint32_t)(p * (uint32_t)CW) & 3u;
                        uint32_t cw[RUNW];
#pragma unroll
                        for (uint32_t i = 0; i < RUNW; ++i) cw[i] = __builtin_amdgcn_alignbyte(craw[i + 1], craw[i], ca);
                        // One group per run: g = this read's group so far (else the run's first window's, when single).
                        // A branch-free pass finds d0, the first valid window that is neither g nor multi-group
                        // (another group, or SENT); windows [0, d0) are tallied at once and the run is cut at d0, which
                        // starts the next iteration (with that group as g, or deferred when SENT).
                        const uint32_t c0 = cw[0] & C::SENT;
                        const uint32_t g = gcur != C::NONE ? gcur : (c0 < G ? c0 : C::NONE);
                        const uint32_t gr = g * C::REP, mr = C::MULTI * C::REP;
                        uint32_t cnt = 0, fo = RUNW, fflags = 0;
                        uint64_t gm = 0, mm = 0;  // bit d: window d is g (local mode) / multi-group (EM)
#pragma unroll
                        for (uint32_t i = 0; i < RUNW; ++i) {
                            const uint32_t vm = spread<CW>((uint32_t)(m >> (PER * i)) & ((1u << PER) - 1u));
                            const uint32_t eg = zero_elems<CW>(cw[i] ^ gr) & vm;
                            const uint32_t em = zero_elems<CW>(cw[i] ^ mr) & vm;
                            const uint32_t ot = vm & ~(eg | em);
                            const bool before = fo == RUNW;
                            const uint32_t below = ot ? ((ot & (0u - ot)) - 1u) : ~0u;  // elements before the first other
                            cnt += before ? (uint32_t)__popc(eg & below) : 0u;
                            if (MODE == KM_LOCAL)
                                gm |= (uint64_t)(CW == 1 ? flags4(eg) : (((eg >> 15) & 1u) | ((eg >> 30) & 2u))) << (PER * i);
                            if (EM)
                                mm |= (uint64_t)(CW == 1 ? flags4(em) : (((em >> 15) & 1u) | ((em >> 30) & 2u))) << (PER * i);
                            fflags = (before && ot) ? ot : fflags;
                            fo = (before && ot) ? i : fo;
                        }
                        const uint32_t d0 = fo == RUNW ? AX_RUN : PER * fo + (uint32_t)__builtin_ctz(fflags) / (8u * CW);
                        const bool cut = d0 < R;
                        const uint32_t Rc = cut ? d0 : R;  // windows tallied in this iteration
                        const uint64_t mRc = Rc >= 64u ? ~0ull : ((1ull << Rc) - 1ull);
                        if (cnt) {
                            double wsum = 0.0;
                            if (MODE == KM_LOCAL) {
                                // one quality for the whole cut run when no base in (j, j + Rc - 1 + k) changes it
                                if (chg_zero(sbase + j + 1u, Rc + k - 2u)) {
                                    int q = (int)qj - 33;
                                    q = q < 0 ? 0 : (q > 41 ? 41 : q);
                                    wsum = (double)cnt * wtab[q];
                                } else {
                                    uint64_t todo = gm & mRc;
                                    while (todo) {
                                        const uint32_t d = (uint32_t)__builtin_ctzll(todo);
                                        todo &= todo - 1;
                                        const uint32_t jj = j + d;
                                        const uint8_t* qb = src.qual + a + jj;
                                        int q = (int)qb[0] - 33;
                                        q = q < 0 ? 0 : (q > 41 ? 41 : q);
                                        wsum += weight(qb, chg_zero(sbase + jj + 1u, k - 1u), (uint32_t)q);
                                    }
                                }
                            }
                            add_count(g, cnt, wsum);
                            if (af < 0) af = (int32_t)g;
                            else if ((int32_t)g != af) ad = 1;
                            gcur = g;
                        }
                        if (EM) {  // multi-group windows of the cut run: the EM histogram
                            uint64_t todo = mm & mRc;
                            while (todo) {
                                const uint32_t d = (uint32_t)__builtin_ctzll(todo);
                                todo &= todo - 1;
                                const uint32_t lo = A.mlo[p + d];
                                atomicAdd(&src.em_mult[lo], 1u);
                                src.em_hi[lo] = A.mhi[lo];
                            }
                        }
                        // next state
                        if (cut) {
                            uint32_t x = cw[0];
#pragma unroll
                            for (uint32_t i = 1; i < RUNW; ++i) x = (fo == i) ? cw[i] : x;
                            const uint32_t cl = (x >> (8u * CW * (d0 % PER))) & C::SENT;
                            uint32_t adv = d0;
                            if (cl == C::SENT) {  // matched bases, but no valid text window there: looked up later
                                if (defer_push(lane, j + d0)) {
                                    adv = d0 + 1u;
                                    st = 1u;
                                } else {
                                    st = 0u;  // the list is full: look that window up now
                                    last_mm = -1;
                                }
                            } else {
                                gcur = cl;  // another group: the next iteration tallies from d0 with it
                                st = 1u;
                            }
                            j += adv;
                            p += adv;
                            verify = false;
                        } else {
                            const bool mism = e < cmpb;  // the run ended at a mismatch (base j + e)
                            if (mism && R < wend - j) last_mm = (int32_t)(j + e);
                            j += R;
                            p += R;
                            verify = false;
                            st = (mism || R == 0u) ? 0u : 1u;
                        }
                        if (j >= wend) st = 2u;
                    }
                }
            }

            // ---- phase 2: the deferred windows of the wave. (a) the Bloom filter, AX_F windows per lane per round
            // trip; the windows it cannot rule out are compacted to the front of the list; (b) those are looked up one
            // per lane (bucket -> fingerprint -> compare with the text -> class)
            ambf[lane] = af;
            ambd[lane] = ad;
            wave_sync();
#if SPEQ_AX_PROBE == 2  // timing probe only (wrong results): no deferred windows
            const uint32_t n2 = 0;
#else
            const uint32_t n2 = min(__builtin_amdgcn_readfirstlane(defn[0]), AX_DEF);
#endif
            for (uint32_t base = 0; base < n2; base += 64u * AX_F) {
                uint32_t ent[AX_F];
                uint64_t hh[AX_F];
                uint64_t fw[AX_F];
#pragma unroll
                for (uint32_t t = 0; t < AX_F; ++t) {
                    const uint32_t idx = base + 64u * t + lane;
                    const uint16_t e16 = idx < n2 ? defl[idx] : AX_VOID;
                    ent[t] = e16 == AX_VOID ? AX_EMPTY : (uint32_t)e16;
                    const uint32_t o = ent[t] & 63u, jj = (ent[t] >> 6) & 1023u;
                    uint64_t ra[NWC];
                    read_words((uint32_t)sbs[o] + jj, ra);
                    hh[t] = ax_hash<NWC>(ra, k);
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
            for (uint32_t base = 0; base < n3; base += 64) {
                const uint32_t idx = base + lane;
                const bool act = idx < n3;
                const uint32_t ent = act ? (uint32_t)defl[idx] : 0u;
                const uint32_t o = ent & 63u, jj = ent >> 6;
                const uint32_t sbo = sbs[o];
                uint64_t ra[NWC];
                read_words(sbo + jj, ra);
                const uint64_t h = ax_hash<NWC>(ra, k);
                uint32_t b = act ? ax_bucket(h, A.nb) : 0u, sl = 0, pp = 0;
                bool pend = act, found = false;
                uint32_t cl = C::SENT;
                while (__ballot(pend) != 0) {
                    const bool c = ax_probe(A, rs_atab, (uint32_t)h, b, sl, pp, pend);
                    const bool cand = pend && c;
                    uint64_t tw[NWC];
                    {
                        const uint32_t toff = cand ? (pp >> 5) * 8u : AX_OOB;
                        uint64_t raw[NWC + 1];
#pragma unroll
                        for (int i = 0; i <= NWC; ++i) {
                            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_t2, toff + 8u * (uint32_t)i, 0, 0);
                            raw[i] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
                        }
#pragma unroll
                        for (int i = 0; i < NWC; ++i) tw[i] = funnel(raw[i], raw[i + 1], 2u * (pp & 31u));
                    }
                    const uint32_t cc = load_class(pp, cand);
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
                                cl = cc;
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
                        const bool uni = chg_zero(sbo + jj + 1u, k - 1u);
                        int q = (int)qb[0] - 33;
                        q = q < 0 ? 0 : (q > 41 ? 41 : q);
                        wgt = weight(qb, uni, (uint32_t)q);
                    }
                    add_count(cl, 1u, wgt);
                    const int32_t old = atomicCAS(&ambf[o], -1, (int32_t)cl);
                    if (old != -1 && old != (int32_t)cl) ambd[o] = 1;
                } else if (EM && found && cl == C::MULTI) {
                    const uint32_t lo = A.mlo[pp];
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
            const int32_t of = __builtin_amdgcn_mov_dpp(af, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]: the mate
            const int32_t od = __builtin_amdgcn_mov_dpp(ad, 0xB1, 0xF, 0xF, false);
            const bool amb_pair = ad || od || (af >= 0 && of >= 0 && af != of);
            if (has && (lane & 1u) == 0u && amb_pair) ++amb;
        } else if (has && ad) {
            ++amb;
        }
    }

#if SPEQ_AX_PROBE == 4 || SPEQ_AX_PROBE == 6  // timing probe only (wrong results): no flush of the counters
    if (t_cnt != 0xFFFFFFFFu) return;
#endif
    // wave sums of the window and ambiguity counters through two LDS words (no shuffle address registers)
    if (lane == 0) {
        defn[2] = 0;
        defn[3] = 0;
    }
    wave_sync();
    if (t_cnt) atomicAdd(&defn[2], t_cnt);
    if (amb) atomicAdd(&defn[3], amb);
    wave_sync();
    const unsigned long long tsum = defn[2], asum = defn[3];
    if (lane == 0) {
        if (tsum) atomicAdd(&out_a[0], tsum);
        if (asum) atomicAdd(&out_a[1], asum);
    }
    if (LDS_HIST) {
        __syncthreads();
        for (uint32_t g = threadIdx.x; g < G; g += AX_THREADS) {
            const unsigned long long x = hA[g];
            if (x) atomicAdd(&gU[g], x);
            if (MODE == KM_LOCAL) {
                const double y = hW[g];
                if (y != 0.0) atomicAdd(&out_w[g], y);
            }
        }
    }
}

template <int MODE, bool PAIRED, bool LDS, bool EM, int NWC, int CW>
void ax_launch_one(const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w) {
    if (lds > 64 * 1024)  // dynamic LDS above 64 KiB must be allowed (occupancy caps pad it)
        HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_ax<MODE, PAIRED, LDS, EM, NWC, CW>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL((k_scan_ax<MODE, PAIRED, LDS, EM, NWC, CW>), dim3(grid), dim3(AX_THREADS), lds, st, A, src, a,
                       w);
}

// NWC = words covering the k - 1 + AX_RUN bases of one compare: 3 (k <= 33), 4 (k <= 65), 6 (k <= 128)
template <int MODE, bool PAIRED, bool LDS, bool EM, int CW>
void ax_launch_nwc(uint32_t k, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w) {
    if (k <= 33) ax_launch_one<MODE, PAIRED, LDS, EM, 3, CW>(A, src, grid, lds, st, a, w);
    else if (k <= 65) ax_launch_one<MODE, PAIRED, LDS, EM, 4, CW>(A, src, grid, lds, st, a, w);
    else ax_launch_one<MODE, PAIRED, LDS, EM, 6, CW>(A, src, grid, lds, st, a, w);
}

template <int MODE, bool PAIRED>
void ax_launch_mode(uint32_t cw, bool lds_hist, uint32_t k, const AxView& A, const UnitSrc& src, uint32_t grid,
                    size_t lds, hipStream_t st, unsigned long long* a, double* w) {
    const bool em = src.em_mult != nullptr;
    if (cw == 1) {  // <= 253 groups: always the LDS histogram
        if (em) ax_launch_nwc<MODE, PAIRED, true, true, 1>(k, A, src, grid, lds, st, a, w);
        else ax_launch_nwc<MODE, PAIRED, true, false, 1>(k, A, src, grid, lds, st, a, w);
    } else if (lds_hist) {
        if (em) ax_launch_nwc<MODE, PAIRED, true, true, 2>(k, A, src, grid, lds, st, a, w);
        else ax_launch_nwc<MODE, PAIRED, true, false, 2>(k, A, src, grid, lds, st, a, w);
    } else {
        if (em) ax_launch_nwc<MODE, PAIRED, false, true, 2>(k, A, src, grid, lds, st, a, w);
        else ax_launch_nwc<MODE, PAIRED, false, false, 2>(k, A, src, grid, lds, st, a, w);
    }
}

}  // namespace

namespace speq {

// Builds the per-k anchor structures of replica d (blocking, on its stream). Returns a table with ok == false when
// k, the group count or the index is outside what the scan supports, or the structures would not fit the free HBM.
AxTable build_ax(speq_device_index* d, uint32_t k) {
    DeviceGuard g(d->device);
    const auto t0 = std::chrono::steady_clock::now();
    AxTable ax;
    const uint64_t n = d->view.n;
    if (k < 1 || k > AX_MAX_K || n >= (1ull << 30) || d->G > AxCls<2>::MAX_G) return ax;
    ax.cw = d->G <= AxCls<1>::MAX_G ? 1u : 2u;
    const uint64_t nw64 = (n + 63) / 64 + 4;
    const uint64_t cls_bytes = ((n + 512) * ax.cw + 15) & ~15ull;
    size_t free_b = 0, total_b = 0;
    HIP_OK(hipMemGetInfo(&free_b, &total_b));
    // cls, mlo, mhi, owner, text2 + tbad, table + filter (bounds)
    const uint64_t need = cls_bytes + (n + 64) * 4 * 3 + nw64 * 24 + n * 12;
    if (need > free_b / 10 * 9) return ax;
    uint32_t* owner = nullptr;
    unsigned long long* d_cnt = nullptr;
    std::vector<void*> mine;  // this table's allocations (tracked by the replica once the table is complete)
    auto cleanup = [&] {
        (void)hipStreamSynchronize(d->stream);
        if (owner) (void)hipFree(owner);
        if (d_cnt) (void)hipFree(d_cnt);
        owner = nullptr;
        d_cnt = nullptr;
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
        alloc(&ax.cls, cls_bytes);
        alloc(reinterpret_cast<void**>(&ax.mlo), (n + 64) * 4);
        alloc(reinterpret_cast<void**>(&ax.mhi), (n + 64) * 4);
        HIP_OK(hipMalloc(&owner, (n + 1) * 4));
        HIP_OK(hipMalloc(&d_cnt, 8));
        HIP_OK(hipMemsetAsync(ax.cls, 0xFF, cls_bytes, d->stream));
        HIP_OK(hipMemsetAsync(owner, 0xFF, (n + 1) * 4, d->stream));
        HIP_OK(hipMemsetAsync(d_cnt, 0, 8, d->stream));
        const DevView v = search_view(d, k);
        const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 16384);
        if (ax.cw == 1)
            hipLaunchKernelGGL(k_ax_classify<1>, dim3(grid), dim3(256), 0, d->stream, v, d->d_text, d->d_tbad, n, k,
                               ax.cls, ax.mlo, ax.mhi, owner, d_cnt);
        else
            hipLaunchKernelGGL(k_ax_classify<2>, dim3(grid), dim3(256), 0, d->stream, v, d->d_text, d->d_tbad, n, k,
                               ax.cls, ax.mlo, ax.mhi, owner, d_cnt);
        HIP_OK(hipGetLastError());
        unsigned long long distinct = 0;
        HIP_OK(hipMemcpyAsync(&distinct, d_cnt, 8, hipMemcpyDeviceToHost, d->stream));
        HIP_OK(hipStreamSynchronize(d->stream));
        ax.distinct = distinct;
        ax.nb = std::max<uint64_t>(1, (uint64_t)((double)distinct * 100.0 / (8.0 * d->ax_load)) + 1);
        ax.nf = std::max<uint64_t>(1, distinct * AX_FILTER_BITS / 64);
        if (ax.nb * 64 >= (1ull << 32) - 64 || ax.nf * 8 >= (1ull << 32) - 64) {
            // the scan addresses the tables with 32-bit buffer offsets: leave this k to the other kernels
            cleanup();
            for (void* q : mine) (void)hipFree(q);
            return AxTable{};
        }
        alloc(&ax.atab, ax.nb * 64);
        alloc(&ax.filt, ax.nf * 8);
        HIP_OK(hipMemsetAsync(ax.atab, 0xFF, ax.nb * 64, d->stream));
        HIP_OK(hipMemsetAsync(ax.filt, 0, ax.nf * 8, d->stream));
        hipLaunchKernelGGL(k_ax_insert, dim3(grid), dim3(256), 0, d->stream, owner, n, d->d_text2, k,
                           reinterpret_cast<unsigned long long*>(ax.atab), ax.nb,
                           reinterpret_cast<unsigned long long*>(ax.filt), ax.nf);
        HIP_OK(hipGetLastError());
        HIP_OK(hipStreamSynchronize(d->stream));
        ax.cls_bytes = cls_bytes;
        ax.bytes = ax.nb * 64 + ax.nf * 8 + cls_bytes + (n + 64) * 8;
        ax.ok = true;
    } catch (...) {
        cleanup();
        for (void* q : mine) (void)hipFree(q);
        throw;
    }
    cleanup();
    for (void* q : mine) d->track(q);
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
    A.mlo = ax->mlo;
    A.mhi = ax->mhi;
    A.atab = reinterpret_cast<const unsigned long long*>(ax->atab);
    A.filt = reinterpret_cast<const unsigned long long*>(ax->filt);
    A.nb = ax->nb;
    A.nf = ax->nf;
    A.n = d->view.n;
    A.t2_bytes = ((d->view.n + 63) / 64 + 4) * 16;
    A.cls_bytes = ax->cls_bytes;
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
    if (mode == KM_GLOBAL) {
        if (paired) ax_launch_mode<KM_GLOBAL, true>(ax->cw, lds_hist, src.k, A, src, grid, lds_launch, st, a, w);
        else ax_launch_mode<KM_GLOBAL, false>(ax->cw, lds_hist, src.k, A, src, grid, lds_launch, st, a, w);
    } else {
        if (paired) ax_launch_mode<KM_LOCAL, true>(ax->cw, lds_hist, src.k, A, src, grid, lds_launch, st, a, w);
        else ax_launch_mode<KM_LOCAL, false>(ax->cw, lds_hist, src.k, A, src, grid, lds_launch, st, a, w);
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace speq
