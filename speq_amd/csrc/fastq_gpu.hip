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

#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses ::memset

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <string>

#include "speq_errors.hpp"

namespace speq {
namespace {

#define FHIP(expr)                                                                                            \
    do {                                                                                                      \
        hipError_t _e = (expr);                                                                               \
        if (_e != hipSuccess) throw DeviceError(std::string("fastq gpu: ") + #expr + ": " + hipGetErrorString(_e)); \
    } while (0)

constexpr uint32_t CHUNK = 256;  // bytes per thread in the newline count

enum : uint32_t { ERR_HEADER = 1u, ERR_PLUS = 2u, ERR_LENGTH = 4u, ERR_LINES = 8u };

__device__ __forceinline__ bool is_space(uint32_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
__device__ __forceinline__ bool is_seq(uint32_t c) { return !is_space(c) && !(c >= '0' && c <= '9'); }

__global__ void k_count_nl(const uint8_t* __restrict__ raw, uint64_t len, uint32_t* __restrict__ counts,
                           uint32_t n_chunks) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    const uint64_t b = (uint64_t)c * CHUNK, e = min(len, b + CHUNK);
    uint32_t cnt = 0;
    for (uint64_t i = b; i < e; ++i) cnt += raw[i] == '\n';
    counts[c] = cnt;
}

__global__ void k_write_nl(const uint8_t* __restrict__ raw, uint64_t len, const uint32_t* __restrict__ offs,
                           uint32_t n_chunks, uint32_t* __restrict__ nl, uint32_t cap) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    const uint64_t b = (uint64_t)c * CHUNK, e = min(len, b + CHUNK);
    uint32_t o = offs[c];
    for (uint64_t i = b; i < e; ++i)
        if (raw[i] == '\n') {
            if (o < cap) nl[o] = (uint32_t)i;
            ++o;
        }
}

struct Rec {
    uint32_t s0, s1, q0, q1;  // raw [begin, end) of the base line and of the quality line
};

// One thread per record of one file: line bounds from the newline table, checks, valid character counts.
__global__ void k_records(const uint8_t* __restrict__ raw, uint64_t len, uint32_t base_off,
                          const uint32_t* __restrict__ nl, const uint32_t* __restrict__ n_nl, uint32_t n,
                          uint32_t slot0, uint32_t slot_stride, Rec* __restrict__ rec, uint64_t* __restrict__ lens,
                          uint32_t* __restrict__ err) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint32_t total = *n_nl;
    auto line_end = [&](uint32_t j) -> uint64_t { return j < total ? nl[j] : len; };  // last line may be open
    if (4u * r + 2u >= total) {  // fewer than three newlines before the quality line
        atomicOr(err, ERR_LINES);
        lens[slot0 + r * slot_stride] = 0;
        rec[slot0 + r * slot_stride] = Rec{0, 0, 0, 0};
        return;
    }
    const uint64_t h = r == 0 ? 0 : (uint64_t)nl[4u * r - 1u] + 1u;
    const uint64_t s0 = line_end(4u * r) + 1u, s1 = line_end(4u * r + 1u);
    const uint64_t p0 = s1 + 1u;
    const uint64_t q0 = line_end(4u * r + 2u) + 1u, q1 = line_end(4u * r + 3u);
    uint64_t se = s1, qe = q1;
    while (se > s0 && raw[se - 1] == '\r') --se;
    while (qe > q0 && raw[qe - 1] == '\r') --qe;
    uint32_t e = 0;
    if (h >= len || raw[h] != '@') e |= ERR_HEADER;
    if (p0 >= len || raw[p0] != '+') e |= ERR_PLUS;
    uint64_t ns = 0, nq = 0;
    for (uint64_t i = s0; i < se; ++i) ns += is_seq(raw[i]);
    for (uint64_t i = q0; i < qe; ++i) nq += !is_space(raw[i]);
    if (ns != nq) e |= ERR_LENGTH;
    if (e) atomicOr(err, e);
    lens[slot0 + r * slot_stride] = e ? 0 : ns;
    rec[slot0 + r * slot_stride] = Rec{(uint32_t)s0 + base_off, (uint32_t)se + base_off, (uint32_t)q0 + base_off,
                                       (uint32_t)qe + base_off};
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

inline uint32_t grid(uint64_t n, uint32_t bs = 256) { return (uint32_t)((n + bs - 1) / bs); }
inline uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

struct Layout {
    uint64_t counts, offs, nl, n_nl, rec, lens, temp, total;
};

Layout layout(uint64_t raw_bytes, uint64_t n_slots, uint64_t n_lines, size_t temp_bytes) {
    Layout L{};
    const uint64_t chunks = raw_bytes / CHUNK + 2;
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

size_t temp_need(uint64_t raw_bytes, uint64_t n_slots) {
    size_t a = 0, b = 0;
    const uint64_t chunks = raw_bytes / CHUNK + 2;
    (void)rocprim::exclusive_scan(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)chunks,
                                  rocprim::plus<uint32_t>());
    (void)rocprim::exclusive_scan(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr, uint64_t(0),
                                  (size_t)(n_slots + 1), rocprim::plus<uint64_t>());
    return std::max(a, b);
}

}  // namespace

size_t fastq_gpu_scratch_bytes(uint64_t raw_bytes, uint64_t records_per_file, bool paired) {
    const uint64_t n_slots = records_per_file * (paired ? 2 : 1);
    return layout(raw_bytes, n_slots, 4 * records_per_file, temp_need(raw_bytes, n_slots)).total;
}

// d_raw holds file 1's block [0, len1) followed by file 2's [len1, len1 + len2) (paired). Writes k_scan's input
// layout: records interleaved (2i, 2i+1) when paired; d_off has n_slots + 1 entries. Asynchronous on `stream`.
void launch_fastq_parse(const uint8_t* d_raw, uint64_t len1, uint64_t len2, uint64_t n, bool paired, void* d_scratch,
                        size_t scratch_bytes, uint8_t* d_seq, uint8_t* d_qual, uint64_t* d_off, uint32_t* d_err,
                        void* stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t n_slots = n * (paired ? 2 : 1);
    const uint64_t raw_max = std::max(len1, len2);
    const size_t tn = temp_need(raw_max, n_slots);
    const Layout L = layout(raw_max, n_slots, 4 * n, tn);
    if (L.total > scratch_bytes) throw std::invalid_argument("fastq gpu: scratch too small");
    if (len1 + len2 >= (uint64_t(1) << 32)) throw std::invalid_argument("fastq gpu: block exceeds 4 GiB");
    uint8_t* base = static_cast<uint8_t*>(d_scratch);
    uint32_t* counts = reinterpret_cast<uint32_t*>(base + L.counts);
    uint32_t* offs = reinterpret_cast<uint32_t*>(base + L.offs);
    uint32_t* nl = reinterpret_cast<uint32_t*>(base + L.nl);
    uint32_t* n_nl = reinterpret_cast<uint32_t*>(base + L.n_nl);
    Rec* rec = reinterpret_cast<Rec*>(base + L.rec);
    uint64_t* lens = reinterpret_cast<uint64_t*>(base + L.lens);
    void* temp = base + L.temp;
    for (int f = 0; f < (paired ? 2 : 1); ++f) {
        const uint8_t* raw = d_raw + (f ? len1 : 0);
        const uint64_t len = f ? len2 : len1;
        const uint32_t chunks = (uint32_t)(len / CHUNK + 1);
        k_count_nl<<<grid(chunks), 256, 0, st>>>(raw, len, counts, chunks);
        FHIP(hipGetLastError());
        size_t need = tn;
        // chunks + 1 entries: the last exclusive sum is the total newline count
        FHIP(hipMemsetAsync(counts + chunks, 0, 4, st));
        FHIP(rocprim::exclusive_scan(temp, need, counts, offs, 0u, (size_t)chunks + 1, rocprim::plus<uint32_t>(), st));
        FHIP(hipMemcpyAsync(n_nl, offs + chunks, 4, hipMemcpyDeviceToDevice, st));
        k_write_nl<<<grid(chunks), 256, 0, st>>>(raw, len, offs, chunks, nl, (uint32_t)(4 * n + 1));
        FHIP(hipGetLastError());
        // record r of file f goes to slot paired ? 2r + f : r; raw offsets of file 2 are made global below
        k_records<<<grid(n), 256, 0, st>>>(raw, len, f ? (uint32_t)len1 : 0u, nl, n_nl, (uint32_t)n,
                                           paired ? (uint32_t)f : 0u, paired ? 2u : 1u, rec, lens, d_err);
        FHIP(hipGetLastError());
    }
    size_t need = tn;
    FHIP(hipMemsetAsync(lens + n_slots, 0, 8, st));
    FHIP(rocprim::exclusive_scan(temp, need, lens, d_off, uint64_t(0), (size_t)(n_slots + 1),
                                 rocprim::plus<uint64_t>(), st));
    k_copy<<<grid(n_slots * 64u), 256, 0, st>>>(d_raw, rec, d_off, (uint32_t)n_slots, d_seq, d_qual);
    FHIP(hipGetLastError());
}

}  // namespace speq
