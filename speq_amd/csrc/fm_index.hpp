// Host-side FM-index of the reference collection, laid out for the HIP scan kernels.
//
// Replaces seqan3::fm_index<dna5, collection> built at /root/reference/src/fm_indexer.cpp:36 over the texts
// [fwd_0, rc_0, fwd_1, rc_1, …] (fm_indexer.cpp:25-33). The layout:
//
//   text   : SA alphabet codes, texts separated by SEP and closed by TERM:
//            T = t_0 SEP t_1 SEP … t_{2R-1} SEP TERM          (TERM=0 < SEP=1 < A=2 < C=3 < G=4 < T=5 < N=6)
//   occ    : five planes (A, C, G, T, N), plane-major [symbol][block]; one 16-B entry per 96 BWT positions
//            {u32 C[s] + rank of s before the block, u32 x3 bitmap of the 96 positions}, so LF(s, i) is that count
//            plus a popcount (C[] is folded in: no per-step table lookup). Plane-major keeps
//            the entries of one symbol for 768 consecutive positions in one 128-B line, so the lo and hi loads of
//            a narrow SA interval hit the same line. The N plane is only touched by windows that contain N
//            (the .dat pass).
//   occ2   : optional 16 two-symbol planes (pairs ab over ACGT, plane 4a+b), same entry format: bit j set iff
//            T[SA[j]-2] T[SA[j]-1] == ab, count = C2[ab] + rank, with C2[ab] = #suffixes < "ab". One gather pair
//            then extends the pattern by TWO bases: interval(abP) = (LF2(ab, lo), LF2(ab, hi)).
//   occ3   : optional 64 three-symbol planes (plane 16a+4b+c), count = C3[abc] + rank with C3[abc] = #suffixes <
//            "abc": one gather pair extends the pattern by THREE bases (same argument as occ2).
//   runs   : 16-B entries over the label-change bitvector B[i] = [label(SA[i]) != label(SA[i-1])],
//            label = group of the text holding suffix SA[i]
//   run_label : group id of every run (u16)
//   lab    : optional u32 per SA position: group (low 16 bits) | min(run_end - i, 65535) (high 16 bits), where
//            run_end is one past the label run holding i. [lo,hi) is single-group iff hi - lo <= that distance, so
//            the classification is one 4-B load (the runs/run_label rank path remains for saturated distances).
//   prefix : for every q-mer over ACGT its SA interval (u32 lo, u32 hi); prefix1 / prefix2 the same for q-1 / q-2
//            (a scan picks the level that leaves k - q' divisible by its widest step)
//
// "All occurrences of a window lie in ONE group" <=> the window's SA interval [lo,hi) holds no label change,
// i.e. run(lo) == run(hi-1). That replaces SeqAn3's locate of every occurrence.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace speq {

enum : uint8_t { SYM_TERM = 0, SYM_SEP = 1, SYM_A = 2, SYM_C = 3, SYM_G = 4, SYM_T = 5, SYM_N = 6, SYM_COUNT = 7 };
constexpr uint32_t OCC_BLOCK = 96;   // BWT positions per occ block
constexpr uint32_t MAX_PREFIX_Q = 13;

// dna5 conversion of an ASCII base (seqan3 dna5 assign_char: ACGT/acgt, U/u -> T, anything else -> N).
inline uint8_t ascii_to_sym(unsigned char ch) {
    switch (ch) {
        case 'A': case 'a': return SYM_A;
        case 'C': case 'c': return SYM_C;
        case 'G': case 'g': return SYM_G;
        case 'T': case 't': case 'U': case 'u': return SYM_T;
        default: return SYM_N;
    }
}
inline uint8_t complement_sym(uint8_t s) {
    switch (s) {
        case SYM_A: return SYM_T;
        case SYM_C: return SYM_G;
        case SYM_G: return SYM_C;
        case SYM_T: return SYM_A;
        default: return s;
    }
}

struct OccEntry {  // 16 B
    uint32_t count;
    uint32_t bits[3];
};

struct FmIndex {
    uint64_t n = 0;               // length of text (incl. separators and terminator)
    uint32_t n_records = 0;
    uint32_t n_texts = 0;
    uint32_t n_groups = 0;
    uint32_t prefix_q = 0;
    std::vector<uint8_t> text;            // n
    std::vector<uint64_t> text_start;     // n_texts + 1 (text t occupies [start[t], start[t+1]-1), SEP at start[t+1]-1)
    std::vector<int32_t> text_group;      // n_texts
    std::vector<int32_t> group_of_rec;    // as given (length >= n_records)
    uint32_t C[SYM_COUNT + 1] = {0};      // C[c] = #symbols < c
    std::vector<OccEntry> occ;            // 5 * n_blocks, entry (s, b) at s * n_blocks + b
    std::vector<OccEntry> occ2;           // 16 * n_blocks or empty
    std::vector<OccEntry> occ3;           // 64 * n_blocks or empty (three-symbol planes, plane 16a + 4b + c)
    std::vector<OccEntry> runs;           // n_blocks
    std::vector<uint16_t> run_label;      // n_runs
    std::vector<uint32_t> lab;            // n or empty
    std::vector<uint32_t> prefix;         // 2 * 4^q
    // Shorter q-mer tables (levels q-1 and q-2, empty when q < 2 / 3): the scan picks the level that leaves a
    // number of remaining symbols divisible by its step width (2 or 3), so no single step is needed.
    std::vector<uint32_t> prefix1, prefix2;
    std::vector<int32_t> sa;              // n (host only, not persisted; empty after load)

    uint64_t n_blocks() const { return n / OCC_BLOCK + 1; }
    uint64_t device_bytes() const;

    // Host LF / rank used by the builder and by tests: LF(sym, i) = C[sym] + #sym in BWT[0, i).
    uint32_t lf(uint8_t sym, uint64_t i) const;
    uint32_t lf2(uint8_t a, uint8_t b, uint64_t i) const;  // two-symbol LF (requires occ2)
    uint32_t lf3(uint8_t a, uint8_t b, uint8_t c, uint64_t i) const;  // three-symbol LF (requires occ3)
    uint32_t rank(uint8_t sym, uint64_t i) const;
    uint32_t run_of(uint64_t i) const;   // index of the label run holding SA position i
    uint64_t run_end(uint64_t i) const;  // one past the last position of the label run holding i
    uint16_t label_at(uint64_t i) const { return run_label[run_of(i)]; }
};

// Builds the index (throws std::invalid_argument / std::runtime_error).
void fm_build(FmIndex& idx, const char* seq, const uint64_t* rec_offsets, uint32_t n_records,
              const int32_t* group_of_rec, uint32_t n_group_entries, uint32_t n_groups, uint32_t prefix_q,
              uint32_t threads, bool pair_steps = false, bool label_table = false, int gpu_device = -1,
              bool triple_steps = false);
// GPU half of fm_build (build_gpu.hip): suffix array, occ/occ2/occ3/runs planes, run labels and label table.
// suffix array of a device text (build_gpu.hip); stream = hipStream_t
void gpu_suffix_sort(const uint8_t* d_text, uint32_t n, uint32_t* d_sa, void* stream, bool timing);
void fm_build_arrays_gpu(FmIndex& idx, int device, bool pair_steps, bool triple_steps, bool label_table,
                         bool timing);
// C3[abc] = #suffixes < "abc" (a, b, c in A..T), from symbol-pair and -triple counts of the text.
void triple_bases(const FmIndex& idx, uint32_t out[64]);

void fm_save(const FmIndex& idx, const std::string& path, const void* header, uint64_t header_len);
void fm_load(FmIndex& idx, const std::string& path, std::vector<uint8_t>* header);
void fm_read_header(const std::string& path, std::vector<uint8_t>& header);

}  // namespace speq
