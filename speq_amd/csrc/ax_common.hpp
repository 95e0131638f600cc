// Device code of the anchor-and-extend read scan (ax_scan.hip: k_scan_ax and the per-k structures): constants, compile-time knobs, hashing of k-mers into the anchor
// table and the Bloom filter, the anchor-table slot resolution and probe chain, bit helpers. DESIGN.md §4e.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "scan_device.hpp"
#include "speq_scan.h"

namespace speq_dev {
// The per-k anchor structures as the scan kernels read them (built by build_ax, ax_scan.hip; passed to both kernels)
struct AxView {
    const u32x4* gran;         // granules {2-bit text, class plane 0, class plane 1} per 32 text positions
    const uint32_t* mlo;       // SA interval start of the multi-group k-mer at a text position (EM)
    const uint32_t* mhi;       // its end, by interval start (EM)
    const unsigned long long* atab;  // (followed, in the same allocation, by the m-mer filter: byte offset mf_off)
    const unsigned long long* filt;
    unsigned long long* stats; // STATS instantiation only: AXS_N counters
    uint64_t nb;               // buckets
    uint64_t nf;               // filter words
    uint64_t n;                // text length
    uint64_t gran_bytes;       // bytes of gran (incl. END padding)
    uint64_t nmf;              // m-mer filter words (0: no m-mer absence proofs)
    uint32_t mf_off;           // byte offset of the m-mer filter from atab (the anchor table's buffer descriptor
                               // covers both, so a lookup iteration loads buckets and m-mer filter words alike)
    uint32_t m;                // m of the m-mer filter (0: off)
    uint32_t mtiles;           // 1: also probe windows whose mismatch is unknown (lane state 6)
    uint32_t G;
};
}  // namespace speq_dev

namespace {

using namespace speq_dev;

// Compile-time knobs (A/B only; every one is run through the parity tests forced to a non-default value by
// tests/test_gpu_ax_knobs.py over `make axknobs` builds), sixteen: SPEQ_AX_DEF_LOCAL, SPEQ_AX_DEF_GLOBAL, SPEQ_AX_WL,
// SPEQ_AX_WPB, SPEQ_AX_SU, SPEQ_AX_SU_LOCAL, SPEQ_AX_MIN_WAVES, SPEQ_AX_MIN_WAVES_LOCAL, SPEQ_AX_REFILL, SPEQ_AX_BLOCKED,
// SPEQ_AX_SPEC_HW, SPEQ_AX_PRIO, SPEQ_AX_PRIO_MIN, SPEQ_AX_P2_MARGIN, SPEQ_AX_MPROOF, SPEQ_AX_MTILES. Measured losers
// of rounds 3-5 (a cuckoo anchor table, lowest / first-claimant representatives, a dynamic tail, generation-weighted
// pools, offset prefetch, speculative runs in global mode, a minimizer-keyed filter, workgroup-shared pools) were
// removed; DESIGN.md §4f-§4g keep their numbers.
constexpr uint32_t AX_MAX_K = 128;    // longest k the scan takes (AX_CAP - k + 1 windows per segment)
constexpr uint32_t AX_CAP = 192;      // bases of a read a lane stages at once (longer reads: segments of AX_CAP bases)
constexpr uint32_t AX_STREAM = AX_CAP + 16;  // staged bases incl. the 16-B alignment slack before the read
constexpr uint32_t AX_CHUNKS = AX_STREAM / 16;
constexpr uint32_t AX_CMP = 160;      // bases a run compares per iteration at most: a 150-bp read in one iteration
constexpr uint32_t AX_CMPW = AX_CMP / 32;        // 2-bit words of one compare
constexpr uint32_t AX_NGR = AX_CMPW + 1;         // granules that cover AX_CMP bases from any offset in the first
constexpr uint32_t AX_CHK = 3;                   // 64-window class chunks of one run (<= AX_CMP - k + 1 windows)
constexpr uint32_t AX_VWW = 4;        // valid-window words per lane (>= AX_CAP - k + 1 windows; 16 B per staged chunk)
#ifndef SPEQ_AX_DEF_LOCAL  // deferred-window entries per wave in local mode (A/B knob)
#define SPEQ_AX_DEF_LOCAL 416
#endif
#ifndef SPEQ_AX_DEF_GLOBAL  // the same in global mode (A/B knob; a multiple of 4)
#define SPEQ_AX_DEF_GLOBAL 864
#endif
// deferred-window entries per wave (u16: lane | window << 6): global mode 864 (7.9 KB per wave: 5 blocks of 4 waves
// per CU); local mode 416, so that its 9.7 KB per wave fit 4 blocks per CU (up to 77 groups). (896 / 448 until round
// 6: 32 entries each gave their 64 B to the owner map's third row, SPEQ_AX_SU = 3, so a workgroup's LDS stayed the same
// — with both, config 3's 50-group workgroups no longer fitted 5 per CU: k = 31 1.44 -> 1.91 ms.)
template <int MODE>
constexpr uint32_t ax_def() {
    return MODE == KM_LOCAL ? SPEQ_AX_DEF_LOCAL : SPEQ_AX_DEF_GLOBAL;
}
static_assert(SPEQ_AX_DEF_GLOBAL % 4 == 0 && SPEQ_AX_DEF_LOCAL % 4 == 0, "u64 counters after the deferred list");
constexpr uint32_t AX_F = 4;          // deferred windows a lane tests against the filter per round trip
constexpr uint32_t AX_EMPTY = 0xFFFFFFFFu;
constexpr uint16_t AX_VOID = 0xFFFFu;  // a deferred-list slot reserved by a lane that then kept its windows
constexpr unsigned long long AX_SLOT_EMPTY = ~0ull;
constexpr uint32_t AX_OOB = 0xFFFFFFF0u;  // buffer offset past every array (n < 2^30)
constexpr uint32_t AX_FILTER_BITS = 16;   // Bloom filter bits per distinct k-mer (3 bits set per k-mer, one 64-bit word)
constexpr uint32_t AX_MP = 4;             // m-mer absence probes per lane per lookup iteration (one per bucket load)
constexpr uint32_t AX_MAX_G = 0xFFFFu;    // groups a slot's 16-bit group field holds
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// class codes: plane 0 = bit 0, plane 1 = bit 1
enum : uint32_t { AX_OWN = 0, AX_MULTI = 1, AX_SENT = 2, AX_END = 3 };

static_assert(AX_STREAM % 16 == 0, "chunks of 16 bases");
static_assert(AX_CAP < 1024, "deferred entries hold the window in 10 bits");
static_assert(AX_CMP % 32 == 0 && AX_CMP <= AX_CAP && 64 * AX_CHK >= AX_CMP, "run geometry");

// per-launch work counters of the diagnostic (STATS) instantiation; bench.py turns them into the kernel's own bytes
enum : uint32_t {
    AXS_WAVE_ITERS = 0,  // phase-1 loop iterations (per wave)
    AXS_LOOKUP_LANES,    // phase-1 lane-iterations that loaded an anchor bucket (64 B)
    AXS_RUN_LANES,       // phase-1 lane-iterations that loaded a run's granules
    AXS_LOOKUP_WAVES,    // phase-1 iterations in which the wave issued the bucket loads
    AXS_RUN_WAVES,       // ... the granule loads
    AXS_RUN_WINDOWS,     // windows a run classified (tallied, multi or skipped as invalid)
    AXS_DEFERRED,        // windows put on the deferred list
    AXS_FILTER_PASS,     // deferred windows the Bloom filter could not rule out
    AXS_P2_PROBES,       // phase-2 bucket loads (lanes)
    AXS_P2_VERIFY,       // phase-2 verifications of a candidate (lanes; HW + 1 granules of 16 B)
    AXS_CHUNKS,          // staged 16-base chunks (16 B of bases + 16 B of qualities each)
    AXS_SEGMENTS,        // staged read segments
    AXS_QBYTES,          // single quality bytes loaded (local mode)
    AXS_RUN_TALLIED,     // windows tallied by runs
    AXS_RUN_GRANULES,    // granules (16 B) loaded by phase-1 runs
    AXS_REFILLS,         // refills (staging of the next pieces of idle lanes; per wave)
    AXS_BUSY_1_4,        // phase-1 wave iterations with 1-4 busy lanes
    AXS_BUSY_5_16,       // ... 5-16
    AXS_BUSY_17_32,      // ... 17-32
    AXS_BUSY_33_64,      // ... 33-64
    AXS_CYC_REFILL,      // shader-clock cycles (s_memtime, summed over waves): refills
    AXS_CYC_LOOKUP,      // ... phase-1 lookup iterations
    AXS_CYC_RUN,         // ... phase-1 run iterations
    AXS_CYC_P2,          // ... phase 2 (deferred windows)
    AXS_CYC_TOTAL,       // ... the whole loop
    AXS_P2_PASSES,       // deferred-window passes (per wave)
    AXS_CYC_P2_FILTER,   // ... the Bloom-filter part of phase 2
    AXS_P2_ROUNDS,       // phase-2 probe rounds of the survivors (per wave; a round is bucket + granule loads)
    AXS_CYC_REF_PRE,     // cycles of refills before the staging loads (unit hand-out, read offsets, chunk prefix sums)
    AXS_CYC_REF_STAGE,   // ... their staging batches (loads + decode)
    AXS_CYC_WAVE_MAX,    // the longest wave's loop cycles (max, not a sum: with AXS_CYC_TOTAL / waves, the imbalance)
    AXS_WAVES,           // waves
    AXS_CYC_GEN0,        // loop cycles summed over the waves of blocks 0-255 (dispatched first: the oldest waves of
    AXS_CYC_GEN1,        // their SIMDs), 256-511, 512-767, 768-1023, and 1024 on
    AXS_CYC_GEN2,
    AXS_CYC_GEN3,
    AXS_CYC_GEN4,
    AXS_N
};
static_assert(AXS_N == SPEQ_AX_STATS_N, "speq_scan.h SPEQ_AX_STATS_N");

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
// slot fingerprint: the hash's low 16 bits (the bucket comes from its high 32)
__host__ __device__ __forceinline__ uint32_t ax_fp(uint64_t h) { return (uint32_t)h & 0xFFFFu; }
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
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

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



// Resolves one anchor bucket (8 slots {pos, fp << 16 | group}) from slot `s` on: the first slot whose fingerprint
// matches (candidate position p, its text's group g) before the first empty slot -> 1; an empty slot first -> 0
// (absent); neither (a full bucket) -> 2 (continue in the next bucket).
__device__ __forceinline__ uint32_t ax_resolve(const u32x4& v0, const u32x4& v1, const u32x4& v2, const u32x4& v3,
                                               uint32_t fp, uint32_t s, uint32_t& slot, uint32_t& p, uint32_t& g) {
    const uint32_t pos[8] = {v0[0], v0[2], v1[0], v1[2], v2[0], v2[2], v3[0], v3[2]};
    const uint32_t fg[8] = {v0[1], v0[3], v1[1], v1[3], v2[1], v2[3], v3[1], v3[3]};
    uint32_t mm = 0, me = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const bool empty = pos[t] == AX_EMPTY;
        me |= (empty ? 1u : 0u) << t;
        mm |= ((!empty && (fg[t] >> 16) == fp) ? 1u : 0u) << t;
    }
    const uint32_t from = s >= 8u ? 0u : ((0xFFu << s) & 0xFFu);
    mm &= from;
    me &= from;
    const uint32_t fm = mm ? (uint32_t)__builtin_ctz(mm) : 8u, fe = me ? (uint32_t)__builtin_ctz(me) : 8u;
    if (fm < fe) {
        uint32_t pp = pos[0], gg = fg[0];
#pragma unroll
        for (int t = 1; t < 8; ++t) {
            pp = fm == (uint32_t)t ? pos[t] : pp;
            gg = fm == (uint32_t)t ? fg[t] : gg;
        }
        p = pp;
        g = gg & 0xFFFFu;
        slot = fm;
        return 1u;
    }
    return fe < 8u ? 0u : 2u;
}

// One probe chain of the anchor table from bucket b, slot s (phase 2): stops at the first fingerprint match (found:
// p, g, s) or at an empty slot (absent); the caller verifies the candidate and resumes at s + 1 after a collision.
__device__ __forceinline__ bool ax_probe(const AxView& A, const __amdgpu_buffer_rsrc_t& rs_atab, uint32_t fp,
                                         uint32_t& b, uint32_t& s, uint32_t& p, uint32_t& g, bool active,
                                         uint32_t& probes) {
    bool found = false, pending = active;
    while (__ballot(pending) != 0) {
        const uint32_t boff = pending ? b * 64u : AX_OOB;
        const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff, 0, 0);
        const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 16u, 0, 0);
        const u32x4 v2 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 32u, 0, 0);
        const u32x4 v3 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 48u, 0, 0);
        if (pending) {
            ++probes;
            uint32_t slot = 0;
            const uint32_t r = ax_resolve(v0, v1, v2, v3, fp, s, slot, p, g);
            if (r == 1u) {
                s = slot;
                found = true;
                pending = false;
            } else if (r == 0u) {
                pending = false;  // absent
            } else {
                b = (b + 1u == (uint32_t)A.nb) ? 0u : b + 1u;
                s = 0;
            }
        }
    }
    return found;
}

// LDS of one wave (persistent lanes). Every lane owns a slot holding the read piece it works on; slot arrays are
// transposed ([word][lane]), so lanes reading their own slots at different offsets never share a bank.
//   codes  u32 [AX_CHUNKS][64]  2-bit bases of the piece from its 16-B-aligned start (slot position 0 = a16)
//   vw     u64 [AX_VWW][64]     valid-window bits, read-relative (window j of the piece at bit j); while staging, the
//                               bad-base bits of the refilling lanes, chunk c in 16 bits of the lane's own word c / 4
//   chg    u16 [AX_CHUNKS][64]  (local) quality-change bits per slot position
//   off0s  u8 [64]              the piece's first base in its slot (a - a16)
//   defl   u16 [ax_def]         deferred windows (lane | window << 6), defn u32[4] counters, ambf/ambd i32[64]
//   wl     u32 [AX_WL]          (local) weight work list: 8-window blocks of runs with varying qualities
//                               (lane | block << 6 | window mask << 11); wlm u32 [64] the lane's run (group | j << 16)
// local mode's factor table in LDS (k_scan_ax): ftab[AX_FTAB] indexed by min(quality byte, 75), entry AX_FONE = 1.0,
// then wtab[QLUT_LEN], within the QTAB_BYTES the launch reserves
constexpr uint32_t AX_FONE = 76u, AX_FTAB = AX_FONE + 1u;
static_assert(8u * (AX_FTAB + QLUT_LEN) <= QTAB_BYTES && AX_FONE - 1u == 33u + 41u + 1u, "ftab + wtab in QTAB_BYTES");
#ifndef SPEQ_AX_WL  // weight work-list entries per wave (A/B knob): the blocks of one round of the weighing pass
#define SPEQ_AX_WL 128
#endif
constexpr uint32_t AX_WL = SPEQ_AX_WL;
static_assert(AX_WL % 64u == 0 && AX_WL >= 64u && AX_WL <= 512u, "work list: 1-8 sub-batches of 64 blocks per round");
#ifndef SPEQ_AX_SU  // staging: stream instructions per load batch, global mode (A/B knob). 3 since round 6: the
#define SPEQ_AX_SU 3   // staging code hoisted out of the refill branch left the registers for it at 5 waves/SIMD
#endif                 // (round 4's 3 spilled 20-36 B per lane); k 65-96 and paired k 33-64 keep 2 (3 spills there)
#ifndef SPEQ_AX_SU_LOCAL  // the same, Phred-weighted mode (4 waves/SIMD, 128 VGPRs; A/B knob)
#define SPEQ_AX_SU_LOCAL 3
#endif
template <int MODE, bool PAIRED, int HW>
constexpr uint32_t ax_su() {
    return MODE == KM_LOCAL ? SPEQ_AX_SU_LOCAL
                            : ((HW == 3 || (PAIRED && HW == 2)) && SPEQ_AX_SU > 2 ? 2u : SPEQ_AX_SU);
}
template <int MODE>
constexpr uint32_t ax_ownb() {  // bytes of the staging owner map (64 per stream instruction of a batch)
    return 64u * (MODE == KM_LOCAL ? SPEQ_AX_SU_LOCAL : SPEQ_AX_SU);
}
template <int MODE>
constexpr uint32_t ax_wave_bytes() {
    static_assert(8u * AX_VWW >= 2u * AX_CHUNKS, "the bad-base bits of a staged piece live in its valid-window words");
    return 4u * AX_CHUNKS * 64u + 8u * AX_VWW * 64u + (MODE == KM_LOCAL ? 2u * AX_CHUNKS * 64u : 0u) +
           64u + 2u * ax_def<MODE>() + 24u + 8u * 64u + (MODE == KM_LOCAL ? 4u * AX_WL + 4u * 64u : 0u) +
           ax_ownb<MODE>();
}

#ifndef SPEQ_AX_WPB  // waves per workgroup of k_scan_ax (A/B knob)
#define SPEQ_AX_WPB 4
#endif
constexpr uint32_t AX_WPB = SPEQ_AX_WPB, AX_THREADS = 64 * SPEQ_AX_WPB;
#ifndef SPEQ_AX_MIN_WAVES  // minimum waves per SIMD the register allocator must allow, global mode, k <= 96 (A/B knob):
#define SPEQ_AX_MIN_WAVES 5   // 5 (96 VGPRs, no spills; LDS fits 5 blocks) is 16 % faster than 4 (r03/ax_variants_w5);
#endif                        // 97 <= k <= 128 stays at most 4 (at 5: 8-24 B of spills per lane)
#ifndef SPEQ_AX_MIN_WAVES_LOCAL  // local (Phred-weighted) mode, every k: 4 (<= 128 VGPRs, no spills; its LDS fits 4
#define SPEQ_AX_MIN_WAVES_LOCAL 4   // blocks per CU up to 77 groups); the instrumented twin 3
#endif
#ifndef SPEQ_AX_REFILL  // idle lanes that trigger a refill (staging of their next pieces) while others still run
#define SPEQ_AX_REFILL 16
#endif
#ifndef SPEQ_AX_BLOCKED  // idle lanes waiting for their deferred windows that trigger the deferred-window pass
#define SPEQ_AX_BLOCKED 16
#endif
#ifndef SPEQ_AX_SPEC_HW  // speculative left runs after an absent lookup whose mismatch is unknown, for HW >= this
#define SPEQ_AX_SPEC_HW 3  // (k > 64 by default; 8 = off), Phred-weighted scans only (A/B knob): k = 70 local -5 % at
#endif                     // 0.1 % errors, -14 % at 0.5 %; global mode +6 % (8 B of spills; profiles/r04/ab_*)
#ifndef SPEQ_AX_PRIO  // 1: waves set their issue priority by the share of their pool still to do (A/B knob)
#define SPEQ_AX_PRIO 1
#endif
#ifndef SPEQ_AX_PRIO_MIN  // ... for static pools of at least this many units (and always for k > 64)
#define SPEQ_AX_PRIO_MIN 384u
#endif
#ifndef SPEQ_AX_MPROOF  // 1: the windows that share an absent window's known mismatch are proven absent by m-mer
#define SPEQ_AX_MPROOF 1  // probes where the m-mer filter allows (lane state 4), not deferred (A/B knob; runtime:
#endif                    // tuning ax_mproof)
#ifndef SPEQ_AX_MTILES  // 1: ... and for an absent window whose mismatch is unknown (lane state 6; A/B knob)
#define SPEQ_AX_MTILES 1
#endif
#ifndef SPEQ_AX_P2_MARGIN  // the deferred-window pass also runs when fewer than this many list entries are free
#define SPEQ_AX_P2_MARGIN 256u  // (A/B knob; a deferral that finds the list full waits for the pass: lane state 3)
#endif
// EM scans and the instrumented twin hold more live state: 4 waves (no spills)
template <int MODE, int HW, bool EM, bool STATS>
constexpr int ax_min_waves() {
    return MODE == KM_LOCAL ? (STATS ? 3 : SPEQ_AX_MIN_WAVES_LOCAL)
                            : ((EM || STATS) ? 4
                                             : (HW >= 4 ? (SPEQ_AX_MIN_WAVES < 4 ? SPEQ_AX_MIN_WAVES : 4)
                                                        : SPEQ_AX_MIN_WAVES));
}

__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {  // ({hi, lo} >> (s & 31))[31:0]
    return __builtin_amdgcn_alignbit(hi, lo, s);
}
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {  // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

}  // namespace
