// Anchor-and-extend read scan with a staging wave per workgroup (k_scan_axq), for gfx950 (MI355X). DESIGN.md §4g.
//
// Same per-window semantics as k_scan_ax (ax_scan.hip; /root/reference/src/fm_scanner.cpp:153-196 global,
// :426-471 local, :665-729 paired), same per-k structures (granules, anchor table, Bloom filter) and the same phase-1
// (lookup / run) and phase-2 (deferred windows) code. What differs is who stages the reads. In k_scan_ax a wave whose
// lanes ran out of work stops all 64 lanes while it loads and decodes their next read pieces: 2-3 dependent HBM round
// trips per refill, 34-49 % of the wave time. Here each workgroup has AXQ_C consumer waves (the scan
// itself) and one STAGER wave that owns the workgroup's pool of units (reads or mate pairs): it cuts them into pieces
// (a read segment of at most AXQ_CAP bases, a mate), loads and decodes them (2-bit codes, bad-base bits, quality-change
// bits, valid-window bits, T) into a ready ring of AXQ_B pieces per consumer wave in LDS, ahead of demand. A consumer
// lane that has finished its piece copies the next one from its wave's ring (a few LDS reads; no memory round trip on
// the consumer's critical path). Units of several pieces (mate pairs, reads longer than AXQ_CAP) may be scanned by
// different lanes: each piece carries a ring record of its unit in LDS {first group, another group seen, pieces left}
// and the lane that finishes the unit's last piece counts its ambiguity (fm_scanner.cpp:183-190, :709-729).
//
// Hand-offs are single-producer / single-consumer rings in LDS: the stager writes records, then publishes the head
// (workgroup-scope release); a consumer reads the head (acquire), copies records, then publishes its tail (release).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>

#include "ax_common.hpp"
#include "device_index.hpp"
#include "scan_device.hpp"
#include "scan_internal.hpp"
#include "speq_scan.h"

namespace {

constexpr uint32_t AXQ_CAP = 160;                       // bases of a piece (one compare of AX_CMP covers it)
constexpr uint32_t AXQ_CHUNKS = (AXQ_CAP + 16) / 16;    // 16-base chunks of a piece incl. alignment slack (11)
constexpr uint32_t AXQ_VWW = 3;                         // valid-window words per piece (>= AXQ_CAP - k + 1 windows)
static_assert(AX_CMP >= AXQ_CAP && 64u * AXQ_VWW >= AXQ_CAP && 8u * AXQ_VWW >= 2u * AXQ_CHUNKS, "piece geometry");
constexpr uint32_t AXQ_C = 4;                           // consumer waves per workgroup (+ one stager wave)
constexpr uint32_t AXQ_THREADS = 64u * (AXQ_C + 1u);
constexpr uint32_t AXQ_B = 32;                          // staged pieces a consumer wave's ready ring holds
constexpr uint32_t AXQ_R = 512;                         // unit ring records per workgroup (multi-piece units in flight)
constexpr uint32_t AXQ_DEF = 768;                       // deferred-window entries per consumer wave
constexpr uint32_t AXQ_SU = 4;                          // stager: stream instructions per load batch
constexpr uint32_t AXQ_SPIN_MAX = 1u << 24;              // waits (s_sleep) without progress before a wave gives up
constexpr uint32_t AXQ_NORING = 0xFFFFu;                // a single-piece unit (ambiguity counted by its lane)
static_assert(AXQ_R >= AXQ_C * (64u + AXQ_B) && AXQ_R < AXQ_NORING, "every unit in flight has its own ring record");
static_assert(AXQ_DEF % 4u == 0u, "u64 counters after the deferred list");

// LDS of one consumer wave (byte offsets; global mode): its lanes' slots as in k_scan_ax (codes, valid-window words,
// piece offsets, deferred list, counters, ambiguity), then its ready ring (AXQ_B records, transposed [field][slot])
// and the ring's control words {head (stager), tail (consumer), done (stager)}
struct AxqLayout {
    static constexpr uint32_t codes = 0;                                   // u32 [AXQ_CHUNKS][64]
    static constexpr uint32_t vw = codes + 4u * AXQ_CHUNKS * 64u;          // u64 [AXQ_VWW][64]
    static constexpr uint32_t off0s = vw + 8u * AXQ_VWW * 64u;             // u8 [64]
    static constexpr uint32_t defl = off0s + 64u;                          // u16 [AXQ_DEF]
    static constexpr uint32_t defn = defl + 2u * AXQ_DEF;                  // u32 [2]
    static constexpr uint32_t wsum = defn + 8u;                            // u64 [2]
    static constexpr uint32_t ambf = wsum + 16u;                           // i32 [64]
    static constexpr uint32_t ambd = ambf + 256u;                          // i32 [64]
    static constexpr uint32_t bcodes = ambd + 256u;                        // u32 [AXQ_CHUNKS][AXQ_B]
    static constexpr uint32_t bvw = bcodes + 4u * AXQ_CHUNKS * AXQ_B;      // u64 [AXQ_VWW][AXQ_B] (staging: bad16)
    static constexpr uint32_t bhdr = bvw + 8u * AXQ_VWW * AXQ_B;           // u32 [AXQ_B]
    static constexpr uint32_t ctl = bhdr + 4u * AXQ_B;                     // u32 [4]
    static constexpr uint32_t bytes = (ctl + 16u + 15u) & ~15u;
};
static_assert(AxqLayout::wsum % 8u == 0u && AxqLayout::vw % 8u == 0u && AxqLayout::bvw % 8u == 0u &&
              AxqLayout::bytes % 16u == 0u, "alignment");
constexpr uint32_t AXQ_OWNB = 64u * AXQ_SU;             // stager's owner map (one batch)
constexpr uint32_t axq_block_bytes() { return AXQ_C * AxqLayout::bytes + 4u * AXQ_R + AXQ_OWNB; }

template <int HW, bool EM, bool STATS>
constexpr int axq_min_waves() {
    return (EM || STATS) ? 4 : (HW >= 4 ? 4 : 5);
}

// Consumer waves w < AXQ_C scan; wave AXQ_C stages. MODE is global (integer tallies): the local mode's per-lane
// quality state does not fit the LDS of four consumer waves and their rings (it stays on k_scan_ax).
template <int MODE, bool PAIRED, bool LDS_HIST, bool EM, int HW, bool STATS>
__global__ __launch_bounds__(AXQ_THREADS, (axq_min_waves<HW, EM, STATS>())) void k_scan_axq(AxView A, UnitSrc src,
                                                                              unsigned long long* __restrict__ out_a,
                                                                              double* __restrict__ out_w) {
    static_assert(MODE == KM_GLOBAL, "k_scan_axq: global mode");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = A.G, k = src.k;
    const uint32_t hist_words = LDS_HIST ? G : 0u;
    const uint32_t hist_bytes = (hist_words * 8u + 15u) & ~15u;
    unsigned long long* hA = reinterpret_cast<unsigned long long*>(smem);
    unsigned char* cbase = smem + hist_bytes;                                // consumer regions
    uint32_t* ring = reinterpret_cast<uint32_t*>(cbase + AXQ_C * AxqLayout::bytes);  // [AXQ_R]
    uint8_t* sownb = reinterpret_cast<uint8_t*>(ring + AXQ_R);                 // [AXQ_OWNB] (stager)
    auto creg = [&](uint32_t c) -> unsigned char* { return cbase + c * AxqLayout::bytes; };

    if (LDS_HIST)
        for (uint32_t i = threadIdx.x; i < hist_words; i += AXQ_THREADS) hA[i] = 0ull;
    for (uint32_t c = threadIdx.x; c < AXQ_C; c += AXQ_THREADS) {
        uint32_t* cw = reinterpret_cast<uint32_t*>(creg(c) + AxqLayout::ctl);
        cw[0] = cw[1] = cw[2] = cw[3] = 0u;
        uint32_t* dn = reinterpret_cast<uint32_t*>(creg(c) + AxqLayout::defn);
        dn[0] = dn[1] = 0u;
        unsigned long long* ws = reinterpret_cast<unsigned long long*>(creg(c) + AxqLayout::wsum);
        ws[0] = ws[1] = 0ull;
    }
    __syncthreads();
    unsigned long long* gU = out_a + 2;
    const uint64_t nu = PAIRED ? src.n_units / 2 : src.n_units;  // units: reads, or mate pairs
    const uint32_t segw = AXQ_CAP - k + 1u;                     // windows per piece
    // diagnostic counters (STATS only; wave-level ones are counted by lane 0)
    uint32_t s_iter = 0, s_lk = 0, s_rn = 0, s_lkw = 0, s_rnw = 0, s_rwin = 0, s_def = 0, s_fp = 0, s_p2 = 0,
             s_p2v = 0, s_ch = 0, s_seg = 0, s_qb = 0, s_tal = 0, s_rg = 0, s_spl = 0, s_b4 = 0, s_b16 = 0, s_b32 = 0,
             s_b64 = 0, s_p2n = 0, s_p2r = 0;
    uint64_t c_ref = 0, c_lk = 0, c_rn = 0, c_p2 = 0, c_p2f = 0, c_rpre = 0, c_rstg = 0, c_t0 = STATS ? clock64() : 0ull, c_s = 0;
    unsigned long long t_stage = 0;  // (stager) passing windows of the staged pieces (T)

    if (wid == AXQ_C) {
        // ======================= the stager wave =======================
        // The workgroup's pool: an equal contiguous share of the units (reads, or mate pairs). Every pass takes up to
        // 64 pieces for the consumers' free ring slots (the consumer with the most room first; a unit may be split
        // over passes and consumers), loads their read offsets, stages their 16-base chunks as one coalesced stream
        // (every lane decodes whole chunks, AXQ_SU x 64 per batch; owners from a byte map + DPP prefix max, as in
        // k_scan_ax), computes each piece's valid-window bits and T, then publishes the consumers' ring heads.
        const uint64_t u_end = (nu * (blockIdx.x + 1u)) / gridDim.x;
        uint64_t cur = (nu * blockIdx.x) / gridDim.x;  // first unit not yet completely staged
        uint32_t pk_next = 0;                          // pieces of unit `cur` staged by earlier passes
        uint32_t cur_rid = AXQ_NORING;                 // its ring record (pk_next > 0)
        uint32_t head[AXQ_C];
#pragma unroll
        for (uint32_t c = 0; c < AXQ_C; ++c) head[c] = 0u;
        uint32_t rctr = 0;  // unit ring records handed out
        uint32_t spins = 0;
        const uint32_t qt = 33u + src.cutoff;  // Phred+33 byte <= qt  <=>  clamp(q, 0, 41) <= cutoff (cutoff < 41)
        const uint32_t qt4 = (qt > 0x7Fu ? 0x7Fu : qt) * 0x01010101u;
        const uint32_t allbad = src.cutoff >= 41u ? 0x80808080u : 0u;  // every window fails the quality filter
        auto nsegs = [&](uint64_t L) -> uint32_t {  // pieces of a read of L bases (a read with no window: one)
            const uint64_t W = L >= k ? L - k + 1u : 0u;
            return W ? (uint32_t)((W + segw - 1u) / segw) : 1u;
        };
        while (cur < u_end) {
            if (STATS) c_s = clock64();
            uint32_t room[AXQ_C], tot = 0;
#pragma unroll
            for (uint32_t c = 0; c < AXQ_C; ++c) {
                uint32_t* cw = reinterpret_cast<uint32_t*>(creg(c) + AxqLayout::ctl);
                const uint32_t tl = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&cw[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                room[c] = AXQ_B - (head[c] - tl);
                tot += room[c];
            }
            if (tot < 16u) {  // the consumers hold AXQ_C * AXQ_B - 16 staged pieces: nothing to do yet
                // (watchdog: a consumer that stopped taking pieces is a bug; leave instead of hanging the GPU —
                // the counts then come out wrong and the parity tests fail)
                if (++spins > AXQ_SPIN_MAX) break;
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            spins = 0;
            // the pass's units: lane l -> unit cur + l, its record bounds and piece counts
            const uint64_t u = cur + lane;
            const bool uv = u < u_end;
            uint64_t o0 = 0, o1 = 0, o2 = 0;
            if (uv) {
                o0 = src.off[PAIRED ? 2u * u : u];
                o1 = src.off[PAIRED ? 2u * u + 1u : u + 1u];
                if (PAIRED) o2 = src.off[2u * u + 2u];
            }
            const uint32_t n1 = uv ? nsegs(o1 - o0) : 0u;
            const uint32_t np = uv ? n1 + (PAIRED ? nsegs(o2 - o1) : 0u) : 0u;
            // pieces -> lanes (scalar): piece P of the pass is {unit lane, piece of the unit, consumer, ring slot}
            uint32_t pu = 0, pkv = 0, pc = 0, psl = 0, prid = AXQ_NORING;
            uint32_t given[AXQ_C];
#pragma unroll
            for (uint32_t c = 0; c < AXQ_C; ++c) given[c] = 0u;
            uint32_t P = 0, ul = 0, pk0 = pk_next, rid = cur_rid;
            const uint32_t nunits = (uint32_t)min<uint64_t>(64u, u_end - cur);
            while (P < 64u && ul < nunits) {
                const uint32_t npu = __builtin_amdgcn_readlane(np, ul);
                uint32_t best = AXQ_C, bestr = 0, bhead = 0;
#pragma unroll
                for (uint32_t c = 0; c < AXQ_C; ++c) {
                    const uint32_t r = room[c] - given[c];
                    if (r > bestr) {
                        bestr = r;
                        best = c;
                        bhead = head[c] + given[c];
                    }
                }
                if (best == AXQ_C) break;
                if (pk0 == 0u) rid = npu > 1u ? (rctr++ % AXQ_R) : AXQ_NORING;
                if (lane == P) {  // (lane P's descriptors)
                    pu = ul;
                    pkv = pk0;
                    pc = best;
                    psl = bhead;
                    prid = rid;
                }
#pragma unroll
                for (uint32_t c = 0; c < AXQ_C; ++c) given[c] += c == best ? 1u : 0u;
                ++P;
                if (++pk0 == npu) {
                    ++ul;
                    pk0 = 0;
                }
            }
            cur += ul;
            pk_next = pk0;
            cur_rid = rid;
            // this lane's piece
            const bool pv = lane < P;
            const uint32_t ulp = pv ? pu : 0u;
            const uint64_t b0 = (uint64_t)__shfl((long long)o0, (int)ulp), b1 = (uint64_t)__shfl((long long)o1, (int)ulp);
            const uint64_t b2 = PAIRED ? (uint64_t)__shfl((long long)o2, (int)ulp) : 0ull;
            const uint32_t n1p = (uint32_t)__shfl((int)n1, (int)ulp), npp = (uint32_t)__shfl((int)np, (int)ulp);
            const bool mate2 = PAIRED && pkv >= n1p;
            const uint32_t seg = mate2 ? pkv - n1p : pkv;
            const uint64_t rb = mate2 ? b1 : b0, re = mate2 ? b2 : b1;
            const uint64_t L = re - rb, W = L >= k ? L - k + 1u : 0u;
            const uint64_t s = (uint64_t)seg * segw;
            const uint32_t sb = (pv && W) ? (uint32_t)min<uint64_t>(L - s, AXQ_CAP) : 0u;
            const uint32_t wend = (pv && W) ? (uint32_t)min<uint64_t>(W - s, segw) : 0u;
            const uint64_t a = rb + s, a16 = a & ~15ull;
            const uint32_t off0 = (uint32_t)(a - a16);
            const uint32_t nch = sb ? (off0 + sb + 15u) / 16u : 0u;
            const uint32_t slot = psl % AXQ_B;
            unsigned char* tr = creg(pv ? pc : 0u);  // the piece's consumer region
            if (pv && pkv == 0u && prid != AXQ_NORING) ring[prid] = (0xFFFFu << 16) | npp;  // {no group, 0, pieces}
            if (STATS) {
                s_ch += nch;
                s_seg += pv ? 1u : 0u;
                c_rpre += clock64() - c_s;
            }
            uint64_t c_b = STATS ? clock64() : 0ull;
            // chunk stream: piece lane o's chunks at [pre_o, pre_o + nch_o)
            uint32_t pre = 0, nch_tot = 0;
#pragma unroll
            for (uint32_t bb = 0; bb < 4; ++bb) {
                const unsigned long long m = __ballot((nch >> bb) & 1u);
                pre += lanes_below(m) << bb;
                nch_tot += (uint32_t)__popcll(m) << bb;
            }
            uint32_t ocarry = 0;  // owner mark of the last chunk of the previous 64
            for (uint32_t c0 = 0; c0 < nch_tot; c0 += 64u * AXQ_SU) {
                uint4 sv[AXQ_SU], qv[AXQ_SU];
                uint32_t own[AXQ_SU], ci[AXQ_SU];
#pragma unroll
                for (uint32_t u2 = 0; u2 < AXQ_SU; ++u2) sownb[64u * u2 + lane] = 0;
                if (nch != 0u && pre >= c0 && pre < c0 + 64u * AXQ_SU) sownb[pre - c0] = (uint8_t)(lane + 1u);
                wave_sync();
                uint32_t mk[AXQ_SU];
#pragma unroll
                for (uint32_t u2 = 0; u2 < AXQ_SU; ++u2) mk[u2] = sownb[64u * u2 + lane];
#pragma unroll
                for (uint32_t u2 = 0; u2 < AXQ_SU; ++u2) {
                    const uint32_t c = min(c0 + 64u * u2 + lane, nch_tot - 1u);
                    uint32_t m = mk[u2];
                    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x111, 0xF, 0xF, false));  // row_shr:1
                    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x112, 0xF, 0xF, false));  // row_shr:2
                    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x114, 0xF, 0xF, false));  // row_shr:4
                    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x118, 0xF, 0xF, false));  // row_shr:8
                    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x142, 0xA, 0xF, false));  // row_bcast:15
                    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x143, 0xC, 0xF, false));  // row_bcast:31
                    m = max(m, ocarry);
                    ocarry = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
                    const uint32_t o = m - 1u;
                    own[u2] = o;
                    ci[u2] = c - (uint32_t)__shfl((int)pre, (int)o);
                    const uint64_t go = (uint64_t)__shfl((long long)a16, (int)o) + 16ull * ci[u2];
                    sv[u2] = *reinterpret_cast<const uint4*>(src.seq + go);
                    qv[u2] = *reinterpret_cast<const uint4*>(src.qual + go);
                }
#pragma unroll
                for (uint32_t u2 = 0; u2 < AXQ_SU; ++u2) {
                    const uint32_t c = c0 + 64u * u2 + lane;
                    const uint32_t sd[4] = {sv[u2].x, sv[u2].y, sv[u2].z, sv[u2].w};
                    const uint32_t qd[4] = {qv[u2].x, qv[u2].y, qv[u2].z, qv[u2].w};
                    uint32_t cw = 0, bad = 0;
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
                    }
                    // the owner piece's consumer ring slot
                    const uint32_t tc = (uint32_t)__shfl((int)pc, (int)own[u2]);
                    const uint32_t ts = (uint32_t)__shfl((int)psl, (int)own[u2]) % AXQ_B;
                    if (c < nch_tot) {
                        unsigned char* t = creg(tc);
                        reinterpret_cast<uint32_t*>(t + AxqLayout::bcodes)[ci[u2] * AXQ_B + ts] = cw;
                        reinterpret_cast<uint16_t*>(t + AxqLayout::bvw)[ci[u2] * AXQ_B + ts] = (uint16_t)bad;
                    }
                }
            }
            wave_sync();
            if (STATS) c_rstg += clock64() - c_b;
            if (pv) {
                // good-base bits of the piece, 16 per chunk from a16 (chunks past it are bad), as 6 dwords
                constexpr uint32_t NOK = (AXQ_CHUNKS + 1u) / 2u;
                uint32_t ok[NOK];
                const uint16_t* b16 = reinterpret_cast<const uint16_t*>(tr + AxqLayout::bvw);
#pragma unroll
                for (uint32_t d = 0; d < NOK; ++d) {
                    const uint32_t lo = 2u * d < nch ? (uint32_t)b16[(2u * d) * AXQ_B + slot] : 0xFFFFu;
                    const uint32_t hi = 2u * d + 1u < nch ? (uint32_t)b16[(2u * d + 1u) * AXQ_B + slot] : 0xFFFFu;
                    ok[d] = ~(lo | (hi << 16));
                }
                // valid windows: AND of k consecutive good bits (doubling), then aligned to the piece's first base
                for (uint32_t len = 1u; len < k;) {
                    const uint32_t sft = min(len, k - len);  // 1 .. 64
                    const uint32_t dw = sft >> 5, bs = sft & 31u;
                    if (dw == 0u) {
#pragma unroll
                        for (uint32_t d = 0; d < NOK; ++d) ok[d] &= alignbit(d + 1u < NOK ? ok[d + 1] : 0u, ok[d], bs);
                    } else if (dw == 1u) {
#pragma unroll
                        for (uint32_t d = 0; d < NOK; ++d)
                            ok[d] &= alignbit(d + 2u < NOK ? ok[d + 2] : 0u, d + 1u < NOK ? ok[d + 1] : 0u, bs);
                    } else {  // sft == 64
#pragma unroll
                        for (uint32_t d = 0; d < NOK; ++d) ok[d] &= d + 2u < NOK ? ok[d + 2] : 0u;
                    }
                    len += sft;
                }
                wave_sync();  // (every lane has read its bad bits before any lane overwrites the region with its words)
                uint32_t* vw32 = reinterpret_cast<uint32_t*>(tr + AxqLayout::bvw);
                uint32_t tcnt = 0;  // T (fm_scanner.cpp:164): the piece's passing windows
#pragma unroll
                for (uint32_t d = 0; d < 2u * AXQ_VWW; ++d) {
                    uint32_t v = alignbit(d + 1u < NOK ? ok[d + 1] : 0u, d < NOK ? ok[d] : 0u, off0);
                    const uint32_t bit0 = 32u * d;
                    v = wend <= bit0 ? 0u : (wend < bit0 + 32u ? v & ((1u << (wend - bit0)) - 1u) : v);
                    tcnt += (uint32_t)__popc(v);
                    vw32[((d >> 1) * AXQ_B + slot) * 2u + (d & 1u)] = v;
                }
                t_stage += tcnt;
                reinterpret_cast<uint32_t*>(tr + AxqLayout::bhdr)[slot] = wend | (off0 << 8) | (prid << 16);
            }
            wave_sync();  // every record of the pass is written before the heads move
#pragma unroll
            for (uint32_t c = 0; c < AXQ_C; ++c) {
                if (given[c] != 0u) {
                    head[c] += given[c];
                    uint32_t* cw = reinterpret_cast<uint32_t*>(creg(c) + AxqLayout::ctl);
                    if (lane == 0) __hip_atomic_store(&cw[0], head[c], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            if (STATS) c_ref += clock64() - c_s;
        }
        // the pool is staged: T into consumer 0's counters (flushed after the final barrier), then `done`
        if (t_stage) atomicAdd(reinterpret_cast<unsigned long long*>(creg(0) + AxqLayout::wsum), t_stage);
        wave_sync();
#pragma unroll
        for (uint32_t c = 0; c < AXQ_C; ++c) {
            uint32_t* cw = reinterpret_cast<uint32_t*>(creg(c) + AxqLayout::ctl);
            if (lane == 0) __hip_atomic_store(&cw[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {
        // ======================= a consumer wave =======================
        unsigned char* wb = creg(wid);
        uint32_t* codes = reinterpret_cast<uint32_t*>(wb + AxqLayout::codes);   // [AXQ_CHUNKS][64]
        uint64_t* vw = reinterpret_cast<uint64_t*>(wb + AxqLayout::vw);         // [AXQ_VWW][64]
        uint8_t* off0s = wb + AxqLayout::off0s;                                   // [64]
        uint16_t* defl = reinterpret_cast<uint16_t*>(wb + AxqLayout::defl);     // [AXQ_DEF]
        uint32_t* defn = reinterpret_cast<uint32_t*>(wb + AxqLayout::defn);     // [2]: entries, survivors
        unsigned long long* wsum = reinterpret_cast<unsigned long long*>(wb + AxqLayout::wsum);  // [2]: T, ambiguous
        int32_t* ambf = reinterpret_cast<int32_t*>(wb + AxqLayout::ambf);       // [64] first counted group
        int32_t* ambd = reinterpret_cast<int32_t*>(wb + AxqLayout::ambd);       // [64] another group seen
        const uint32_t* bcodes = reinterpret_cast<const uint32_t*>(wb + AxqLayout::bcodes);
        const uint64_t* bvw = reinterpret_cast<const uint64_t*>(wb + AxqLayout::bvw);
        const uint32_t* bhdr = reinterpret_cast<const uint32_t*>(wb + AxqLayout::bhdr);
        uint32_t* ctl = reinterpret_cast<uint32_t*>(wb + AxqLayout::ctl);        // head, tail, done
        // k_scan_ax's names for this kernel's piece geometry (the phase-1 / phase-2 code below is k_scan_ax's)
        constexpr uint32_t AX_DEF = AXQ_DEF;
        constexpr uint32_t AX_CHUNKS = AXQ_CHUNKS;
        constexpr uint32_t AX_VWW = AXQ_VWW;
        uint16_t* chg = nullptr;         // (local mode only)
        double2* qtab = nullptr;
        double* wtab = nullptr;
        double* hW = nullptr;
        uint32_t* wl = nullptr;
        uint32_t* wlm = nullptr;
        (void)chg;
        (void)qtab;
        (void)wtab;
        (void)hW;
        (void)wl;
        (void)wlm;
        const __amdgpu_buffer_rsrc_t rs_gran =
            __builtin_amdgcn_make_buffer_rsrc((void*)A.gran, (short)0, (int)(uint32_t)A.gran_bytes, 0x00020000);
        const __amdgpu_buffer_rsrc_t rs_atab =
            __builtin_amdgcn_make_buffer_rsrc((void*)A.atab, (short)0, (int)(uint32_t)(A.nb * 64u), 0x00020000);
        const __amdgpu_buffer_rsrc_t rs_filt =
            __builtin_amdgcn_make_buffer_rsrc((void*)A.filt, (short)0, (int)(uint32_t)(A.nf * 8u), 0x00020000);
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
        // Phred weight of the window whose first quality byte is src.qual[qo]. fm_scanner.cpp:454 divides 1 by the lut
        // values of its k qualities in turn: a window of one quality takes that quotient from wtab (bit-exact); any
        // other window is the product of the k reciprocals qtab[q].y = fl(1 / lut[q]), within 3 k 2^-53 of the
        // reference's quotient (relative). Qualities are read as the aligned dwords that hold them.
        auto weight = [&](uint64_t qo, bool uniform) -> double {
            const uintptr_t ad = reinterpret_cast<uintptr_t>(src.qual + qo);
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)ad & 3u;
            auto qof = [](uint32_t byte) -> uint32_t {
                const int q = (int)byte - 33;
                return q < 0 ? 0u : (q > 41 ? 41u : (uint32_t)q);
            };
            if (uniform) {
                if (STATS) s_qb += 1u;
                return wtab[qof((wp[0] >> (8u * sh)) & 0xFFu)];
            }
            const uint32_t nd = (sh + k + 3u) >> 2;
            double x = 1.0;
            for (uint32_t t = 0; t < nd; ++t) {
                const uint32_t w = wp[t];
    #pragma unroll
                for (uint32_t b = 0; b < 4u; ++b) {
                    const uint32_t idx = 4u * t + b;  // the window's base idx - sh
                    const double f = qtab[qof((w >> (8u * b)) & 0xFFu)].y;
                    x = (idx >= sh && idx < sh + k) ? x * f : x;
                }
            }
            if (STATS) s_qb += k;
            return x;
        };
        // the summed weights of the windows t (bits of mask, t < 8) of a block whose first window's first quality byte is
        // src.qual[qo] (k >= 8): every window t is L_t M R_t with M the product of the reciprocals of bytes 7 .. k - 1
        // (shared by the 8 windows), L_t of bytes t .. 6 and R_t of bytes k .. k + t - 1, so k + 21 products weigh 8
        // windows instead of 8 k. Any product tree over k factors rounds k - 1 times: the bound of weight() holds.
        // Only the dwords that hold a byte of a window in the mask are read (none past the read's last quality byte).
        auto weight8 = [&](uint64_t qo, uint32_t mask) -> double {
            const uintptr_t ad = reinterpret_cast<uintptr_t>(src.qual + qo);
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)ad & 3u;
            auto qinv = [&](uint32_t byte) -> double {
                const int q = (int)(byte & 0xFFu) - 33;
                return qtab[q < 0 ? 0 : (q > 41 ? 41 : q)].y;
            };
            const uint32_t tmax = 31u - (uint32_t)__builtin_clz(mask);  // the last window of the block to weigh
            const uint32_t a0 = wp[0], a1 = wp[1], a2 = sh >= 2u ? wp[2] : 0u;
            const uint32_t l03 = __builtin_amdgcn_alignbyte(a1, a0, sh), l47 = __builtin_amdgcn_alignbyte(a2, a1, sh);
            const uint32_t rs = sh + k, rsh = rs & 3u, rlast = rsh + tmax;  // right bytes k .. k + tmax - 1
            const uint32_t* rp = wp + (rs >> 2);
            const uint32_t c0 = tmax >= 1u ? rp[0] : 0u, c1 = rlast > 4u ? rp[1] : 0u, c2 = rlast > 8u ? rp[2] : 0u;
            const uint32_t r03 = __builtin_amdgcn_alignbyte(c1, c0, rsh), r47 = __builtin_amdgcn_alignbyte(c2, c1, rsh);
            double M = 1.0;
            for (uint32_t t = (sh + 7u) >> 2; t <= (sh + k - 1u) >> 2; ++t) {
                const uint32_t w = wp[t];
    #pragma unroll
                for (uint32_t b = 0; b < 4u; ++b) {
                    const uint32_t idx = 4u * t + b;
                    const double f = qinv(w >> (8u * b));
                    M = (idx >= sh + 7u && idx < sh + k) ? M * f : M;
                }
            }
            double L[8];
            L[7] = 1.0;
    #pragma unroll
            for (int t = 6; t >= 0; --t) L[t] = qinv((t < 4 ? l03 : l47) >> (8 * (t & 3))) * L[t + 1];
            double MR = M, sum = 0.0;
    #pragma unroll
            for (uint32_t t = 0; t < 8u; ++t) {
                sum += ((mask >> t) & 1u) ? L[t] * MR : 0.0;
                if (t < 7u) MR *= qinv((t < 4u ? r03 : r47) >> (8u * (t & 3u)));
            }
            if (STATS) s_qb += k + tmax;
            return sum;
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

        bool hasdef = false;       // deferred windows of this lane's piece are in the wave's list
        int32_t af = -1, ad = 0;   // ambiguity state of the piece: first counted group, another group seen
        bool havepiece = false;    // a piece was taken and is not finalized yet
        uint32_t rid = AXQ_NORING; // its unit's ring record (units of several pieces)
        uint32_t tail = 0;         // pieces taken from the wave's ready ring (wave-uniform)
        uint32_t spins = 0;        // consecutive waits for the stager
        // a piece is complete (its windows and deferred windows counted): fold its ambiguity into its unit's
        // (fm_scanner.cpp:183-190; a pair's mates: :709-729). Ring record {first group : 16, seen : 1, pieces left : 15}
        auto finalize = [&]() {
            if (rid == AXQ_NORING) {
                if (ad) atomicAdd(&wsum[1], 1ull);
                return;
            }
            uint32_t old = __hip_atomic_load(&ring[rid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), nw = 0;
            for (;;) {
                const uint32_t first = old >> 16;
                uint32_t seen = ((old >> 15) & 1u) | (ad ? 1u : 0u), f2 = first;
                if (af >= 0) {
                    if (first == 0xFFFFu) f2 = (uint32_t)af;
                    else if (first != (uint32_t)af) seen = 1u;
                }
                nw = (f2 << 16) | (seen << 15) | ((old & 0x7FFFu) - 1u);
                const uint32_t prev = atomicCAS(&ring[rid], old, nw);
                if (prev == old) break;
                old = prev;
            }
            if ((old & 0x7FFFu) == 1u && ((nw >> 15) & 1u)) atomicAdd(&wsum[1], 1ull);  // the unit's last piece
        };
        // ---- phase-1 state of the current piece
        uint32_t wend = 0;         // windows of the piece
        uint32_t off0 = 0;         // first base of the piece in the slot
        uint64_t ta = 0;           // first base of the piece in seq/qual (local mode; other lanes read it by a shuffle)
        uint32_t j = 0;
        uint32_t st = 2u;          // 0: look window j up, 1: extend from text position p, 2: idle, 3: wait for the
                                   // deferred-window pass (its deferral found the list full), then look window j up
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
        uint32_t sp = 0;  // pending windows [sp, sp + k - 2] of the piece; 0: none
        // defers the valid windows of [lo, hi] (hi - lo <= 127; hi < lo: none) of this lane's piece; when the list has
        // no room: the reserved slots are voided, the lane waits for the deferred-window pass (st 3) and false
        auto defer_range = [&](uint32_t lo, uint32_t hi) -> bool {
            if (hi + 1u <= lo) return true;
            const uint32_t span = hi + 1u - lo;
            uint64_t dm0 = vbits(lane, lo), dm1 = span > 64u ? vbits(lane, lo + 64u) : 0ull;
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

        for (;;) {
            // ================= housekeeping (wave-uniform decisions) =================
            const unsigned long long idle = __ballot(st == 2u);
            const unsigned long long blk = __ballot(st >= 2u && hasdef);
            const unsigned long long busy = ~idle;
            // (a lane whose deferral found the list full, st 3, counts as blocked: the list then holds more than AX_DEF
            // entries, so this pass runs, and the lane looks its window up again afterwards)
            const bool p2 = blk != 0 && ((uint32_t)__popcll(blk) >= SPEQ_AX_BLOCKED || busy == 0 ||
                                         (uint32_t)__builtin_amdgcn_readfirstlane(defn[0]) + (uint32_t)SPEQ_AX_P2_MARGIN > AX_DEF);
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
            // ---- staged pieces for the lanes that are done (idle, no deferred windows pending), in lane order: copied
            // from the wave's ready ring into the lanes' slots (no memory round trip)
            const bool ready = st == 2u && !hasdef;
            const unsigned long long rdy = __ballot(ready);
            if (rdy != 0 && ((uint32_t)__popcll(rdy) >= SPEQ_AX_REFILL || busy == 0)) {
                const uint32_t h = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                const uint32_t n = min(h - tail, (uint32_t)__popcll(rdy));
                if (n != 0u) {
                    if (STATS) s_spl += lane == 0 ? 1u : 0u;
                    const uint32_t rank = lanes_below(rdy);
                    if (ready && rank < n) {
                        if (havepiece) finalize();
                        const uint32_t slot = (tail + rank) % AXQ_B;
    #pragma unroll
                        for (uint32_t c = 0; c < AXQ_CHUNKS; ++c) codes[c * 64u + lane] = bcodes[c * AXQ_B + slot];
    #pragma unroll
                        for (uint32_t w = 0; w < AXQ_VWW; ++w) vw[w * 64u + lane] = bvw[w * AXQ_B + slot];
                        const uint32_t hd = bhdr[slot];
                        wend = hd & 0xFFu;
                        off0 = (hd >> 8) & 15u;
                        rid = hd >> 16;
                        off0s[lane] = (uint8_t)off0;
                        havepiece = true;
                        af = -1;
                        ad = 0;
                        j = 0;
                        sp = 0;
                        verify = false;
                        resume = false;
                        last_mm = -1;
                        st = wend > 0u ? 0u : 2u;
                    }
                    tail += n;
                    spins = 0;
                    wave_sync();  // the records are read before their ring slots are handed back
                    if (lane == 0) __hip_atomic_store(&ctl[1], tail, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (STATS) c_ref += clock64() - c_s;
                    continue;
                }
            }
            if (busy == 0) {
                // every lane idle without deferred windows (else phase 2 ran above) and nothing staged: the end, or wait
                if (__builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&ctl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0u &&
                    (uint32_t)__builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == tail)
                    break;
                if (++spins > AXQ_SPIN_MAX) break;  // (watchdog, as the stager's)
                __builtin_amdgcn_s_sleep(1);
                if (STATS) c_ref += clock64() - c_s;
                continue;
            }
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
            const bool want_lk = __ballot(st == 0u) != 0, want_rn = __ballot(st == 1u) != 0;
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
                const uint32_t boff2 = boff + 32u;
                const u32x4 q0 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff, 0, 0);
                const u32x4 q1 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff + 16u, 0, 0);
                const u32x4 q2 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff2, 0, 0);
                const u32x4 q3 = __builtin_amdgcn_raw_buffer_load_b128(rs_atab, boff2 + 16u, 0, 0);
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
                            if (defer_range(j + 1u, dend)) {
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
                        // the run goes on after it, its first k bases still to be compared
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
                    // whole wave, at most 4 blocks of every lane per pass (a lane sums a block's windows, one atomic)
                    uint32_t nzb = 0;
                    if (wl_pend) {
    #pragma unroll
                        for (uint32_t c = 0; c < AX_CMPW; ++c)
    #pragma unroll
                            for (uint32_t b = 0; b < 4u; ++b)
                                nzb |= (((ownc[c] >> (8u * b)) & 0xFFu) != 0u ? 1u : 0u) << (4u * c + b);
                        wlm[lane] = wl_g | (wl_j << 16);
                    }
                    while (__ballot(nzb != 0u) != 0) {
                        const uint32_t take = min((uint32_t)__popc(nzb), AX_WL_TAKE);
                        uint32_t pre = 0, tot = 0;
    #pragma unroll
                        for (uint32_t b = 0; b < 3u; ++b) {
                            const unsigned long long m = __ballot(((take >> b) & 1u) != 0u);
                            pre += lanes_below(m) << b;
                            tot += (uint32_t)__popcll(m) << b;
                        }
                        for (uint32_t t = 0; t < take; ++t) {
                            const uint32_t blk = (uint32_t)__builtin_ctz(nzb);
                            nzb &= nzb - 1u;
                            const uint32_t c = blk >> 2;
                            const uint32_t oc = c == 0u ? ownc[0] : (c == 1u ? ownc[1] : (c == 2u ? ownc[2] : (c == 3u ? ownc[3] : ownc[4])));
                            wl[pre + t] = lane | (blk << 6) | (((oc >> (8u * (blk & 3u))) & 0xFFu) << 11);
                        }
                        wave_sync();
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
        if (havepiece) finalize();  // (every lane is idle with no deferred window left)
    }
    const uint64_t c_tot = STATS ? clock64() - c_t0 : 0ull;
    __syncthreads();
    if (wid < AXQ_C && lane == 0) {
        const unsigned long long* ws = reinterpret_cast<const unsigned long long*>(creg(wid) + AxqLayout::wsum);
        const unsigned long long tsum = ws[0], asum = ws[1];
        if (tsum) atomicAdd(&out_a[0], tsum);
        if (asum) atomicAdd(&out_a[1], asum);
    }
    if (STATS) {
        const uint64_t sv[AXS_N] = {s_iter, s_lk, s_rn, s_lkw, s_rnw, s_rwin, s_def, s_fp, s_p2, s_p2v, s_ch, s_seg,
                                    s_qb, s_tal, s_rg, s_spl, s_b4, s_b16, s_b32, s_b64,
                                    lane == 0 ? c_ref : 0ull, lane == 0 ? c_lk : 0ull, lane == 0 ? c_rn : 0ull,
                                    lane == 0 ? c_p2 : 0ull, lane == 0 && wid < AXQ_C ? c_tot : 0ull, s_p2n,
                                    lane == 0 ? c_p2f : 0ull, s_p2r, lane == 0 ? c_rpre : 0ull,
                                    lane == 0 ? c_rstg : 0ull, 0ull, lane == 0 && wid < AXQ_C ? 1ull : 0ull, 0ull, 0ull,
                                    0ull, 0ull, 0ull};
#pragma unroll
        for (uint32_t i = 0; i < AXS_N; ++i)
            if (sv[i]) atomicAdd(&A.stats[i], (unsigned long long)sv[i]);
        if (lane == 0 && wid < AXQ_C) {
            atomicMax(&A.stats[AXS_CYC_WAVE_MAX], (unsigned long long)c_tot);
            atomicAdd(&A.stats[AXS_CYC_GEN0 + min(blockIdx.x / 256u, 4u)], (unsigned long long)c_tot);
        }
    }
    if (LDS_HIST) {
        for (uint32_t g = threadIdx.x; g < G; g += AXQ_THREADS) {
            const unsigned long long x = hA[g];
            if (x) atomicAdd(&gU[g], x);
        }
    }
    (void)out_w;
}

template <bool PAIRED, bool LDS, bool EM, int HW, bool STATS>
void axq_launch_one(const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                    unsigned long long* a, double* w, uint32_t n_cus) {
    const void* fn = reinterpret_cast<const void*>(&k_scan_axq<KM_GLOBAL, PAIRED, LDS, EM, HW, STATS>);
    if (lds > 64 * 1024) HIP_OK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    static std::mutex mu;
    static size_t cached_lds = 0;
    static int cached_blocks = 0;
    int per_cu = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (cached_lds != lds || cached_blocks == 0) {
            int nb = 0;
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, AXQ_THREADS, lds));
            cached_lds = lds;
            cached_blocks = std::max(nb, 1);
        }
        per_cu = cached_blocks;
    }
    grid = std::min<uint32_t>(grid, (uint32_t)per_cu * n_cus);
    hipLaunchKernelGGL((k_scan_axq<KM_GLOBAL, PAIRED, LDS, EM, HW, STATS>), dim3(grid), dim3(AXQ_THREADS), lds, st, A,
                       src, a, w);
}

template <bool PAIRED, bool LDS, bool EM, bool STATS>
void axq_launch_hw(uint32_t k, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds, hipStream_t st,
                   unsigned long long* a, double* w, uint32_t n_cus) {
    if (k <= 32) axq_launch_one<PAIRED, LDS, EM, 1, STATS>(A, src, grid, lds, st, a, w, n_cus);
    else if (k <= 64) axq_launch_one<PAIRED, LDS, EM, 2, STATS>(A, src, grid, lds, st, a, w, n_cus);
    else if (k <= 96) axq_launch_one<PAIRED, LDS, EM, 3, STATS>(A, src, grid, lds, st, a, w, n_cus);
    else axq_launch_one<PAIRED, LDS, EM, 4, STATS>(A, src, grid, lds, st, a, w, n_cus);
}

template <bool PAIRED>
void axq_launch_mode(bool lds_hist, uint32_t k, const AxView& A, const UnitSrc& src, uint32_t grid, size_t lds,
                     hipStream_t st, unsigned long long* a, double* w, uint32_t n_cus) {
    const bool em = src.em_mult != nullptr;
    if (A.stats != nullptr && lds_hist && !em) {
        axq_launch_hw<PAIRED, true, false, true>(k, A, src, grid, lds, st, a, w, n_cus);
        return;
    }
    if (lds_hist) {
        if (em) axq_launch_hw<PAIRED, true, true, false>(k, A, src, grid, lds, st, a, w, n_cus);
        else axq_launch_hw<PAIRED, true, false, false>(k, A, src, grid, lds, st, a, w, n_cus);
    } else {
        if (em) axq_launch_hw<PAIRED, false, true, false>(k, A, src, grid, lds, st, a, w, n_cus);
        else axq_launch_hw<PAIRED, false, false, false>(k, A, src, grid, lds, st, a, w, n_cus);
    }
}

}  // namespace

namespace speq {

// k_scan_axq for a global-mode read scan (launch_ax decides; ax_scan.hip). Returns false when it cannot take it.
bool launch_axq(speq_device_index* d, bool paired, const AxView& A, const UnitSrc& src, hipStream_t st,
                unsigned long long* a, double* w) {
    if (src.k > AXQ_CAP - 32u) return false;  // (pieces of at least 32 windows)
    const bool lds_hist = d->G <= LDS_HIST_MAX_G;
    const size_t lds = (((lds_hist ? d->G : 0u) * 8u + 15u) & ~15u) + axq_block_bytes();
    if (lds > 160u * 1024u) return false;
    const uint64_t units = paired ? src.n_units / 2 : src.n_units;
    uint64_t blocks = (units + 64u * AXQ_C - 1u) / (64u * AXQ_C);
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, d->grid_blocks_ax));
    const uint32_t slots = d->n_cus * d->ax_generations;
    if (paired) axq_launch_mode<true>(lds_hist, src.k, A, src, (uint32_t)blocks, lds, st, a, w, slots);
    else axq_launch_mode<false>(lds_hist, src.k, A, src, (uint32_t)blocks, lds, st, a, w, slots);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace speq
