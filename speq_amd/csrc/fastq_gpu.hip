// FASTQ record parsing on the GPU for simple four-line blocks (speq_scan_fastq's fast path).
//
// The host reader cuts record-aligned blocks; when every record of a block has the four-line layout (header '@',
// bases, '+', qualities of the same raw length), the raw bytes go to HBM as they are and are parsed here, instead of
// being split by host threads: newline positions by a chunked count + scan + write, one thread per record for the
// line bounds and the checks, a scan of the record lengths, and one wave per record to copy bases and qualities into
// the (seq, qual, offsets) layout k_scan reads. The grammar is the host parser's (fastq_stream.cpp): trailing '\r'
// trimmed, blanks and digits dropped from base lines, blanks dropped from quality lines, and a record whose base and
// quality counts differ is an error (reported through d_err; the host raises it when the scan finishes).
// Replaces the per-record split of seqan3::sequence_file_input (/root/reference/src/fm_scanner.cpp:138-141).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "speq_errors.hpp"

namespace speq {
namespace {

#define FHIP(expr)                                                                                            \
    do {                                                                                                      \
        hipError_t _e = (expr);                                                                               \
        if (_e != hipSuccess) throw DeviceError(std::string("fastq gpu: ") + #expr + ": " + hipGetErrorString(_e)); \
    } while (0)

// Newline scan: each thread owns one 16-byte aligned window of the block's text (coalesced dwordx4 loads), each
// workgroup 256 windows = 4 KiB.
constexpr uint32_t NL_THREADS = 256, NL_WIN = 16, NL_SPAN = NL_THREADS * NL_WIN;

enum : uint32_t { ERR_HEADER = 1u, ERR_PLUS = 2u, ERR_LENGTH = 4u, ERR_LINES = 8u };

__device__ __forceinline__ bool is_space(uint32_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
__device__ __forceinline__ bool is_seq(uint32_t c) { return !is_space(c) && !(c >= '0' && c <= '9'); }

// bit i set when byte i of w is '\n' (exact: the 7-bit add cannot carry across bytes)
__device__ __forceinline__ uint32_t nl4(uint32_t w) {
    const uint32_t y = w ^ 0x0a0a0a0au;
    const uint32_t t = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);
    return (((t >> 7) & 0x01010101u) * 0x01020408u) >> 24;
}

// '\n' mask of the window starting at byte a (16-aligned) of `base`, restricted to [begin, end)
__device__ __forceinline__ uint32_t nl_mask(const uint8_t* __restrict__ base, uint64_t a, uint64_t begin,
                                            uint64_t end) {
    if (a >= end) return 0;
    const uint4 v = *reinterpret_cast<const uint4*>(base + a);  // the buffer is padded past the text
    uint32_t m = nl4(v.x) | (nl4(v.y) << 4) | (nl4(v.z) << 8) | (nl4(v.w) << 12);
    if (a < begin) m &= 0xffffu << (uint32_t)(begin - a);
    if (end - a < 16) m &= (1u << (uint32_t)(end - a)) - 1u;
    return m;
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}

// Newlines per workgroup span; counts[g] for g < n_groups.
__global__ __launch_bounds__(NL_THREADS) void k_count_nl(const uint8_t* __restrict__ base, uint64_t a0,
                                                         uint64_t begin, uint64_t end,
                                                         uint32_t* __restrict__ counts) {
    __shared__ uint32_t part[NL_THREADS / 64];
    const uint64_t a = a0 + (uint64_t)blockIdx.x * NL_SPAN + (uint64_t)threadIdx.x * NL_WIN;
    uint32_t c = (uint32_t)__popc(nl_mask(base, a, begin, end));
#pragma unroll
    for (uint32_t d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63u) == 0) part[threadIdx.x / 64u] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// Positions (relative to base) of the newlines, in order, from the exclusive sums of k_count_nl.
__global__ __launch_bounds__(NL_THREADS) void k_write_nl(const uint8_t* __restrict__ base, uint64_t a0,
                                                         uint64_t begin, uint64_t end,
                                                         const uint32_t* __restrict__ offs,
                                                         uint32_t* __restrict__ nl, uint32_t cap) {
    __shared__ uint32_t part[NL_THREADS / 64];
    const uint64_t a = a0 + (uint64_t)blockIdx.x * NL_SPAN + (uint64_t)threadIdx.x * NL_WIN;
    uint32_t m = nl_mask(base, a, begin, end);
    const uint32_t c = (uint32_t)__popc(m);
    const uint32_t incl = wave_incl_sum(c);
    const uint32_t w = threadIdx.x / 64u;
    if ((threadIdx.x & 63u) == 63u) part[w] = incl;
    __syncthreads();
    uint32_t o = offs[blockIdx.x] + incl - c;
    for (uint32_t i = 0; i < w; ++i) o += part[i];
    while (m) {
        const uint32_t b = (uint32_t)__ffs(m) - 1u;
        m &= m - 1u;
        if (o < cap) nl[o] = (uint32_t)(a + b);
        ++o;
    }
}

struct Rec {
    uint32_t s0, s1, q0, q1;  // [begin, end) of the base line and of the quality line, relative to base
};

// Characters of [b, e) that pass the filter (bases: not blank, not a digit; qualities: not blank), one wave.
template <bool SEQ>
__device__ __forceinline__ uint64_t wave_count(const uint8_t* __restrict__ base, uint64_t b, uint64_t e,
                                               uint32_t lane) {
    uint64_t n = 0;
    for (uint64_t i0 = b; i0 < e; i0 += 64u) {
        const uint64_t i = i0 + lane;
        const uint32_t c = i < e ? base[i] : (uint32_t)' ';
        n += (uint64_t)__popcll(__ballot(i < e && (SEQ ? is_seq(c) : !is_space(c))));
    }
    return n;
}

// One wave per record of one file (lines 4r .. 4r+3 of the block): line bounds from the newline table, the
// four-line checks, filtered character counts. A record that does not pass sets err (lens 0).
__global__ __launch_bounds__(256) void k_records(const uint8_t* __restrict__ base, uint64_t begin, uint64_t end,
                                                 const uint32_t* __restrict__ nl,
                                                 const uint32_t* __restrict__ n_nl, uint32_t n, uint32_t slot0,
                                                 uint32_t slot_stride, Rec* __restrict__ rec,
                                                 uint64_t* __restrict__ lens, uint32_t* __restrict__ err) {
    const uint32_t r = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    if (r >= n) return;
    const uint32_t total = *n_nl;
    const uint32_t slot = slot0 + r * slot_stride;
    if (4u * r + 2u >= total) {  // fewer than three newlines before the quality line
        if (lane == 0) {
            atomicOr(err, ERR_LINES);
            lens[slot] = 0;
            rec[slot] = Rec{0, 0, 0, 0};
        }
        return;
    }
    auto line_end = [&](uint32_t j) -> uint64_t { return j < total ? nl[j] : end; };  // last line may be open
    const uint64_t h = r == 0 ? begin : (uint64_t)nl[4u * r - 1u] + 1u;
    const uint64_t s0 = line_end(4u * r) + 1u, s1 = line_end(4u * r + 1u);
    const uint64_t p0 = s1 + 1u;
    const uint64_t q0 = line_end(4u * r + 2u) + 1u, q1 = line_end(4u * r + 3u);
    uint64_t se = s1, qe = q1;
    while (se > s0 && base[se - 1] == '\r') --se;
    while (qe > q0 && base[qe - 1] == '\r') --qe;
    uint32_t e = 0;
    if (h >= end || base[h] != '@') e |= ERR_HEADER;
    // the third line must open with '+', and the second must not (the host grammar would take it as the separator)
    if (p0 >= end || base[p0] != '+' || (s0 < s1 && base[s0] == '+')) e |= ERR_PLUS;
    const uint64_t ns = wave_count<true>(base, s0, se, lane), nq = wave_count<false>(base, q0, qe, lane);
    if (ns != nq) e |= ERR_LENGTH;
    if (lane == 0) {
        if (e) atomicOr(err, e);
        lens[slot] = e ? 0 : ns;
        rec[slot] = Rec{(uint32_t)s0, (uint32_t)se, (uint32_t)q0, (uint32_t)qe};
    }
}

// One wave per record slot: copy (and compact) the base and quality characters.
__global__ void k_copy(const uint8_t* __restrict__ raw, const Rec* __restrict__ rec, const uint64_t* __restrict__ off,
                       uint32_t n_slots, uint8_t* __restrict__ seq, uint8_t* __restrict__ qual) {
    const uint32_t slot = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    if (slot >= n_slots) return;
    const Rec R = rec[slot];
    const uint64_t o = off[slot], n = off[slot + 1] - o;
    if (n == 0) return;
    const uint64_t sl = R.s1 - R.s0, ql = R.q1 - R.q0;
    if (sl == n && ql == n) {  // no character to drop: straight coalesced copy
        for (uint64_t i = lane; i < n; i += 64u) {
            seq[o + i] = raw[R.s0 + i];
            qual[o + i] = raw[R.q0 + i];
        }
        return;
    }
    for (int part = 0; part < 2; ++part) {
        const uint64_t b = part ? R.q0 : R.s0, e = part ? R.q1 : R.s1;
        uint8_t* dst = (part ? qual : seq) + o;
        uint64_t w = 0;
        for (uint64_t i0 = b; i0 < e; i0 += 64u) {
            const uint64_t i = i0 + lane;
            const uint32_t c = i < e ? raw[i] : ' ';
            const bool keep = i < e && (part ? !is_space(c) : is_seq(c));
            const uint64_t m = __ballot(keep);
            const uint32_t before = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (keep && w + before < n) dst[w + before] = (uint8_t)c;
            w += (uint64_t)__popcll(m);
        }
    }
}

// Total parsed bases of the batch, accumulated for the stream statistics.
__global__ void k_add_total(const uint64_t* __restrict__ off_end, unsigned long long* __restrict__ total) {
    atomicAdd(total, (unsigned long long)*off_end);
}

// Exclusive scan of n items (the newline counts of a block's 4 KiB spans; the record lengths), out of place, in two
// launches: each 2,048-item tile's sum, then every tile scanned after adding the sums of the tiles before it (a block
// adds those itself: a FASTQ block has at most a few dozen tiles). Until round 6 rocPRIM's scan: its 480 kernel
// instantiations made this file's code object load 3-5 ms (and up to 12 ms more under the start-up's contention)
// where the scan needs two kernels.
constexpr uint32_t SCAN_THREADS = 256, SCAN_ITEMS = 8, SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

template <typename T>
__global__ __launch_bounds__(SCAN_THREADS) void k_tile_sums(const T* __restrict__ in, uint64_t n, T* __restrict__ sums) {
    __shared__ T part[SCAN_THREADS / 64];
    const uint64_t t0 = (uint64_t)blockIdx.x * SCAN_TILE;
    T x = 0;
    for (uint32_t i = threadIdx.x; i < SCAN_TILE; i += SCAN_THREADS) x += t0 + i < n ? in[t0 + i] : T(0);
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o);
    if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = 0;
        for (uint32_t w = 0; w < SCAN_THREADS / 64; ++w) t += part[w];
        sums[blockIdx.x] = t;
    }
}

template <typename T>
__global__ __launch_bounds__(SCAN_THREADS) void k_tile_scan(const T* __restrict__ in, T* __restrict__ out, uint64_t n,
                                                            const T* __restrict__ sums) {
    __shared__ T part[SCAN_THREADS / 64];
    __shared__ T base;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    // the sums of the tiles before this one
    T b = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += SCAN_THREADS) b += sums[i];
    for (int o = 32; o > 0; o >>= 1) b += __shfl_down(b, o);
    if (lane == 0) part[w] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = 0;
        for (uint32_t q = 0; q < SCAN_THREADS / 64; ++q) t += part[q];
        base = t;
    }
    __syncthreads();
    // this thread's SCAN_ITEMS consecutive items
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    T v[SCAN_ITEMS];
    T tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < SCAN_ITEMS; ++j) {
        v[j] = i0 + j < n ? in[i0 + j] : T(0);
        tot += v[j];
    }
    // exclusive prefix of the thread totals: within the wave, then over the waves
    T x = tot;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    __syncthreads();  // (part is reused)
    if (lane == 63) part[w] = x;
    __syncthreads();
    T run = base + x - tot;
    for (uint32_t q = 0; q < w; ++q) run += part[q];
#pragma unroll
    for (uint32_t j = 0; j < SCAN_ITEMS; ++j) {
        if (i0 + j < n) out[i0 + j] = run;
        run += v[j];
    }
}

inline uint64_t scan_tiles(uint64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

// out[i] = in[0] + ... + in[i - 1]; `sums` holds scan_tiles(n) items
template <typename T>
void exclusive_scan(const T* in, T* out, uint64_t n, T* sums, hipStream_t st) {
    if (n == 0) return;
    const uint32_t tiles = (uint32_t)scan_tiles(n);
    k_tile_sums<T><<<tiles, SCAN_THREADS, 0, st>>>(in, n, sums);
    FHIP(hipGetLastError());
    k_tile_scan<T><<<tiles, SCAN_THREADS, 0, st>>>(in, out, n, sums);
    FHIP(hipGetLastError());
}

inline uint32_t grid(uint64_t n, uint32_t bs = 256) { return (uint32_t)((n + bs - 1) / bs); }
inline uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

struct Layout {
    uint64_t counts, offs, nl, n_nl, rec, lens, temp, total;
};

// workgroups of the newline scan over [begin, begin + len) (first window aligned down to 16 bytes)
inline uint64_t nl_groups(uint64_t len) { return (len + NL_WIN) / NL_SPAN + 1; }

Layout layout(uint64_t raw_bytes, uint64_t n_slots, uint64_t n_lines, size_t temp_bytes) {
    Layout L{};
    const uint64_t chunks = nl_groups(raw_bytes) + 2;
    uint64_t p = 0;
    L.counts = p; p = align16(p + chunks * 4);
    L.offs = p; p = align16(p + chunks * 4);
    L.nl = p; p = align16(p + (n_lines + 2) * 4);
    L.n_nl = p; p = align16(p + 16);
    L.rec = p; p = align16(p + n_slots * sizeof(Rec));
    L.lens = p; p = align16(p + (n_slots + 1) * 8);
    L.temp = p; p = align16(p + temp_bytes);
    L.total = p;
    return L;
}

// the scans' tile sums (8 B each: the record-length scan's are u64)
size_t temp_need(uint64_t raw_bytes, uint64_t n_slots) {
    const uint64_t chunks = nl_groups(raw_bytes) + 2;
    return (size_t)std::max(scan_tiles(chunks), scan_tiles(n_slots + 1)) * 8;
}

}  // namespace

namespace {
// Packed host reads (pipeline_submit_packed): one byte per base, bits 0-1 the base (A C G T = 0..3), bits 2-7 the
// Phred value clamped to [0, 41] (phred42), 63 for a base that is not A/C/G/T/U (dna5 N). Back to the (seq, qual)
// bytes the scan kernels read: 'A' 'C' 'G' 'T' or 'N', quality 33 + q. 16 bases per thread, coalesced.
__global__ void k_unpack_bases(const uint8_t* __restrict__ packed, uint64_t n, uint8_t* __restrict__ seq,
                               uint8_t* __restrict__ qual) {
    const uint64_t nv = (n + 15) / 16;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = v * 16;
        if (a + 16 <= n) {
            const uint4 x = *reinterpret_cast<const uint4*>(packed + a);
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
            uint32_t so[4], qo[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t c = w[i] & 0x03030303u, q = (w[i] >> 2) & 0x3F3F3F3Fu;
                const uint32_t letters = __builtin_amdgcn_perm(0u, 0x54474341u, c);  // "ACGT" by code
                const uint32_t y = q ^ 0x3F3F3F3Fu;  // zero byte <=> N
                const uint32_t isn = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
                const uint32_t nm = (isn >> 7) * 0xFFu;  // 0xFF in every N byte
                so[i] = (letters & ~nm) | (0x4E4E4E4Eu & nm);
                qo[i] = ((q + 0x21212121u) & ~nm) | (0x21212121u & nm);
            }
            *reinterpret_cast<uint4*>(seq + a) = make_uint4(so[0], so[1], so[2], so[3]);
            *reinterpret_cast<uint4*>(qual + a) = make_uint4(qo[0], qo[1], qo[2], qo[3]);
        } else {
            for (uint64_t i = a; i < n; ++i) {
                const uint32_t b = packed[i], q = b >> 2;
                seq[i] = q == 63u ? 'N' : "ACGT"[b & 3u];
                qual[i] = (uint8_t)(q == 63u ? 33u : 33u + q);
            }
        }
    }
}

// Global-mode packing (pipeline_submit_packed3): 2 bits per base (A C G T) in u64 words of 32 bases, then one "bad"
// bit per base (not A/C/G/T/U, or Phred <= cutoff) in u32 words. A bad base comes back as 'N' and a good one with the
// largest phred42 quality: window validity (fm_scanner.cpp:162) is unchanged, and global mode reads nothing else.
__global__ void k_unpack_bases3(const uint64_t* __restrict__ codes, const uint32_t* __restrict__ bad, uint64_t n,
                                uint8_t* __restrict__ seq, uint8_t* __restrict__ qual) {
    const uint64_t nw = (n + 31) / 32;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = codes[w];
        const uint32_t b = bad[w];
        uint32_t so[8], qo[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t cb = (uint32_t)(c >> (8 * i)) & 0xFFu;  // four 2-bit codes
            const uint32_t c4 = (cb & 3u) | (((cb >> 2) & 3u) << 8) | (((cb >> 4) & 3u) << 16) | ((cb >> 6) << 24);
            const uint32_t bb = (b >> (4 * i)) & 0xFu;
            const uint32_t nm = ((bb * 0x00204081u) & 0x01010101u) * 0xFFu;  // 0xFF in every bad byte
            const uint32_t letters = __builtin_amdgcn_perm(0u, 0x54474341u, c4);
            so[i] = (letters & ~nm) | (0x4E4E4E4Eu & nm);
            qo[i] = 0x4A4A4A4Au;  // 'J' = 33 + 41
        }
        const uint64_t a = w * 32;
        if (a + 32 <= n) {
            *reinterpret_cast<uint4*>(seq + a) = make_uint4(so[0], so[1], so[2], so[3]);
            *reinterpret_cast<uint4*>(seq + a + 16) = make_uint4(so[4], so[5], so[6], so[7]);
            *reinterpret_cast<uint4*>(qual + a) = make_uint4(qo[0], qo[1], qo[2], qo[3]);
            *reinterpret_cast<uint4*>(qual + a + 16) = make_uint4(qo[4], qo[5], qo[6], qo[7]);
        } else {
            for (uint64_t i = a; i < n; ++i) {
                seq[i] = (uint8_t)(so[(i - a) >> 2] >> (8 * ((i - a) & 3u)));
                qual[i] = 0x4Au;
            }
        }
    }
}
}  // namespace

void launch_unpack_bases3(const uint64_t* d_codes, const uint32_t* d_bad, uint64_t n, uint8_t* d_seq, uint8_t* d_qual,
                          void* stream) {
    if (n == 0) return;
    const uint64_t nw = (n + 31) / 32;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nw + 255) / 256, 8192);
    hipLaunchKernelGGL(k_unpack_bases3, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), d_codes, d_bad, n,
                       d_seq, d_qual);
    FHIP(hipGetLastError());
}

void launch_unpack_bases(const uint8_t* d_packed, uint64_t n, uint8_t* d_seq, uint8_t* d_qual, void* stream) {
    if (n == 0) return;
    const uint64_t nv = (n + 15) / 16;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nv + 255) / 256, 8192);
    hipLaunchKernelGGL(k_unpack_bases, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), d_packed, n, d_seq,
                       d_qual);
    FHIP(hipGetLastError());
}

size_t fastq_gpu_scratch_bytes(uint64_t raw_bytes, uint64_t records_per_file, bool paired) {
    const uint64_t n_slots = records_per_file * (paired ? 2 : 1);
    return layout(raw_bytes, n_slots, 4 * records_per_file, temp_need(raw_bytes, n_slots)).total;
}

// d_raw holds file 1's block [0, len1) followed by file 2's [len1, len1 + len2) (paired), and at least 16 readable
// bytes after them. Writes k_scan's input layout: records interleaved (2i, 2i+1) when paired; d_off has n_slots + 1
// entries; the batch's base count is added to *d_total_bases. Asynchronous on `stream`.
void launch_fastq_parse(const uint8_t* d_raw, uint64_t len1, uint64_t len2, uint64_t n, bool paired, void* d_scratch,
                        size_t scratch_bytes, uint8_t* d_seq, uint8_t* d_qual, uint64_t* d_off, uint32_t* d_err,
                        uint64_t* d_total_bases, void* stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t n_slots = n * (paired ? 2 : 1);
    const uint64_t raw_max = std::max(len1, len2);
    const size_t tn = temp_need(raw_max, n_slots);
    const Layout L = layout(raw_max, n_slots, 4 * n, tn);
    if (L.total > scratch_bytes) throw std::invalid_argument("fastq gpu: scratch too small");
    if (len1 + len2 >= (uint64_t(1) << 32)) throw std::invalid_argument("fastq gpu: block exceeds 4 GiB");
    if (reinterpret_cast<uintptr_t>(d_raw) & 15u) throw std::invalid_argument("fastq gpu: raw buffer not 16-aligned");
    uint8_t* sb = static_cast<uint8_t*>(d_scratch);
    uint32_t* counts = reinterpret_cast<uint32_t*>(sb + L.counts);
    uint32_t* offs = reinterpret_cast<uint32_t*>(sb + L.offs);
    uint32_t* nl = reinterpret_cast<uint32_t*>(sb + L.nl);
    uint32_t* n_nl = reinterpret_cast<uint32_t*>(sb + L.n_nl);
    Rec* rec = reinterpret_cast<Rec*>(sb + L.rec);
    uint64_t* lens = reinterpret_cast<uint64_t*>(sb + L.lens);
    void* temp = sb + L.temp;
    for (int f = 0; f < (paired ? 2 : 1); ++f) {
        const uint64_t begin = f ? len1 : 0, end = begin + (f ? len2 : len1);
        const uint64_t a0 = begin & ~uint64_t(NL_WIN - 1);
        const uint32_t groups = (uint32_t)((end - a0 + NL_SPAN - 1) / NL_SPAN + (end == a0));
        k_count_nl<<<groups, NL_THREADS, 0, st>>>(d_raw, a0, begin, end, counts);
        FHIP(hipGetLastError());
        // groups + 1 entries: the last exclusive sum is the total newline count
        FHIP(hipMemsetAsync(counts + groups, 0, 4, st));
        exclusive_scan<uint32_t>(counts, offs, (uint64_t)groups + 1, static_cast<uint32_t*>(temp), st);
        FHIP(hipMemcpyAsync(n_nl, offs + groups, 4, hipMemcpyDeviceToDevice, st));
        k_write_nl<<<groups, NL_THREADS, 0, st>>>(d_raw, a0, begin, end, offs, nl, (uint32_t)(4 * n + 1));
        FHIP(hipGetLastError());
        // record r of file f goes to slot paired ? 2r + f : r
        k_records<<<grid(n * 64u), 256, 0, st>>>(d_raw, begin, end, nl, n_nl, (uint32_t)n, paired ? (uint32_t)f : 0u,
                                                 paired ? 2u : 1u, rec, lens, d_err);
        FHIP(hipGetLastError());
    }
    FHIP(hipMemsetAsync(lens + n_slots, 0, 8, st));
    exclusive_scan<uint64_t>(lens, d_off, n_slots + 1, static_cast<uint64_t*>(temp), st);
    k_copy<<<grid(n_slots * 64u), 256, 0, st>>>(d_raw, rec, d_off, (uint32_t)n_slots, d_seq, d_qual);
    FHIP(hipGetLastError());
    if (d_total_bases) {
        k_add_total<<<1, 1, 0, st>>>(d_off + n_slots, reinterpret_cast<unsigned long long*>(d_total_bases));
        FHIP(hipGetLastError());
    }
}

}  // namespace speq

namespace speq {
// Loads this translation unit's code object onto the current device (HIP loads a code object at the first use of
// one of its kernels: 30-55 ms for the scan kernels' on the first launch of a `speq scan` run; speq_device_warmup).
void warm_module_fastq_gpu() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_count_nl));
}
}  // namespace speq
