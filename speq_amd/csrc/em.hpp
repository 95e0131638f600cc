// EM refinement state shared by the device half (scan_kernels.hip) and the host half (em.cpp) of the C ABI.
//
// The reference re-reads and re-searches every read in every EM iteration (/root/reference/src/fm_scanner.cpp:
// 1069-1453, loops :248-279). A window's contribution, (c_i p_i / n_i) / sum_j (c_j p_j / n_j), depends only on the
// per-group occurrence counts c of its k-mer -- the per-window factor (temp_acc :1099 / qavg :1188-1193) cancels --
// and c depends only on the window's SA interval. So one GPU pass records {interval -> multiplicity} for windows
// whose occurrences span >= 2 groups (single-group windows are the U[g] counters), and every EM iteration is a sweep
// over that compact histogram.
#pragma once
#include <cstdint>
#include <vector>

#include "capi_internal.hpp"

struct speq_device_index;

struct speq_em {
    const speq_index* idx = nullptr;
    speq_device_index* dev = nullptr;
    uint64_t n = 0;      // SA positions
    uint32_t G = 0;
    uint32_t* d_mult = nullptr;  // device: per SA position, # multi-group windows whose interval starts there
    uint32_t* d_hi = nullptr;    // device: end of that interval
    bool finalized = false;
    uint64_t n_intervals = 0;  // distinct multi-group intervals recorded (rows before equal rows are merged)
    uint64_t n_entries = 0;    // their (group, count) entries
    // CSR rows, one per distinct (group, count) content of the intervals (equal rows merged, multiplicities summed):
    // multiplicity, then (group, count) entries by group id
    std::vector<uint64_t> row_mult;
    std::vector<uint64_t> row_ptr;
    std::vector<uint32_t> col_group;
    std::vector<uint32_t> col_count;
};

namespace speq {
// Builds the CSR rows (host, multi-threaded) from the positions that start a recorded interval, ascending, with their
// multiplicities and interval ends (compacted on the GPU by speq_em_finalize): one row per interval, in position order.
void em_build_rows(speq_em& em, const uint32_t* lo, const uint32_t* mult, const uint32_t* hi, uint64_t m);
// Merges rows of equal content (em.cpp); em_build_rows calls it
void merge_equal_rows(speq_em& em);
}  // namespace speq
