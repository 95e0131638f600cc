// The device replica of an index (speq_device_index, opaque in include/speq_scan.h) and its per-k structures.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "scan_device.hpp"

namespace speq_dev {
struct AxView;  // ax_common.hpp
}

using speq_dev::DevView;

namespace speq {
// Per-k structures of the anchor-and-extend scan (ax_scan.hip).
struct AxTable {
    void* gran = nullptr;      // per 32 text positions {2-bit text, class plane 0, class plane 1} (see ax_scan.hip)
    uint32_t* mlo = nullptr;   // SA interval start of the multi-group k-mer at a text position (EM scans only: built
    uint32_t* mhi = nullptr;   // on the first EM scan of k, ensure_ax_em) / its end, indexed by its interval start
    void* atab = nullptr;      // anchor table: 64-B buckets of 8 {representative position, fingerprint, group} slots
    void* filt = nullptr;      // blocked Bloom filter of the distinct k-mers (one 64-bit word per k-mer, 3 bits)
    uint64_t nb = 0;           // buckets (64 B, 8 slots, linear probing)
    uint32_t load = 0;         // load factor the table was built at (percent)
    uint64_t nf = 0;           // filter words
    uint64_t nmf = 0;          // m-mer filter words (after the nb buckets in atab's allocation; 0: none)
    uint32_t m = 0;            // m of the m-mer filter (0: none)
    uint64_t gran_bytes = 0;
    uint64_t distinct = 0;     // distinct k-mers of the texts
    uint64_t bytes = 0;        // device bytes of the structures
    double build_ms = 0.0;
    bool ok = false;
    bool transient = false;    // !ok only because the free HBM was short at build time (ensure_ax retries)
};
}  // namespace speq

struct speq_device_index {
    int device = 0;
    DevView view{};
    std::vector<void*> allocs;  // every device allocation of the replica, freed by the destructor
    template <typename T>
    T* track(T* p) {
        if (p) allocs.push_back((void*)p);
        return p;
    }
    ~speq_device_index();
    uint8_t* d_text = nullptr;
    uint64_t* d_text_start = nullptr;
    int32_t* d_text_group = nullptr;
    double* d_qlut = nullptr;
    std::vector<uint64_t> text_start;  // host copy (ref pass window sums)
    uint32_t n_texts = 0;
    uint32_t G = 0;
    hipStream_t stream = nullptr;
    bool timing = false;
    uint32_t blocks_per_cu = 0;   // tuning: 0 = as many as registers/LDS allow; else pad LDS to cap occupancy
    uint32_t grid_blocks = 8192;  // tuning: upper bound of the grid
    uint32_t ilp = 1;             // tuning: windows per lane searched concurrently (1 or 2; profiles/r01/sweep_ilp)
    uint32_t ilp_local = 1;       // the same for Phred-weighted scans (NWIN = 2 is slower there: sweep_local.jsonl)
    uint32_t n_cus = 256;
    const uint2* prefix_level[3] = {nullptr, nullptr, nullptr};  // q-mer tables for q, q-1, q-2
    const uint4* sparse_rank[3] = {nullptr, nullptr, nullptr};    // their sparse forms (see prefix_lookup)
    const uint2* sparse_iv[3] = {nullptr, nullptr, nullptr};
    uint64_t present[3] = {0, 0, 0};                              // distinct q-mers per level
    uint64_t prefix_words[3] = {0, 0, 0};                         // u32 words of the dense tables
    std::mutex sparse_mu;                                         // the sparse forms are built on first use
    bool sparse_built = false;
    bool fastq_gpu = true;        // tuning "fastq_gpu_parse": parse simple four-line FASTQ blocks on the GPU
    uint32_t stream_lanes = 3;    // tuning "stream_lanes": compute streams per pipeline (batches scanned concurrently)
    int sparse_choice = 0;        // tuning "sparse_prefix": 0 dense (default), 1 sparse, -1 sparse when < 1/8 of
                                  // the codes occur. Dense wins: the sparse form saves fabric bytes but adds a
                                  // dependent load to every window (cfg 2: 4.63 -> 5.39 ms, sweep_sparse.jsonl)
    int prefix_choice = -1;       // tuning "prefix_level": -1 = by k (view_for_k), 0..2 = force q - level
    uint32_t base_q = 0;          // the index's prefix_q
    bool kmer_table = true;       // tuning "kmer_table": scans of k <= 31 look windows up in a per-k k-mer table
    uint32_t ilp_kt = 0;          // tuning "ilp_kt": windows per lane of k-mer-table scans (1, 2 or 4; 0 = auto:
                                  // 1 for compact tables, 2 for 16-B-slot tables, profiles/r01/ab_notes.txt)
    uint32_t blocks_per_cu_kt = 0;  // tuning "blocks_per_cu_kt": blocks_per_cu of k-mer-table scans (default: no cap)
    uint32_t grid_blocks_kt = 8192;  // tuning "grid_blocks_kt": grid cap of k-mer-table scans (cfg 2: 8192 +4.6 % over
                                     // 16384; fewer is slower: sweep_kt_grid.txt)
    bool kt_pipeline = true;        // tuning "kt_pipeline": k_scan_kt (software-pipelined) for ilp_kt <= 2 read scans
    bool kt_compact = true;       // tuning "kt_compact": 8-B-slot tables for k <= 23 (smaller, mostly L2-resident)
    uint32_t kt_load8 = 35;       // tuning "kt_load8": load factor of compact tables, percent (35-42 best at cfg 2,
                                  // sweep_kt_load8_sgpr.jsonl)
    uint32_t kt_slots = 2;        // tuning "kt_slots": table slots per distinct k-mer (load factor 1/kt_slots .. 2/kt_slots)
    struct KmerTable {
        uint4* table = nullptr;
        uint64_t buckets = 0, distinct = 0;
        double build_ms = 0.0;
        bool compact = false;   // 8-B slots (k <= KT8_MAX_K), `buckets` of 64 B, any count
        uint2* multi = nullptr; // compact: {lo, hi} per multi-group k-mer
        uint64_t bytes = 0;     // device bytes of the table (+ multi array)
    };
    std::mutex kt_mu;                        // the first scan with a new k builds its table
    std::map<uint32_t, KmerTable> ktabs;     // k -> table (kept until the replica closes)
    // anchor-and-extend scan (ax_scan.hip)
    uint64_t* d_text2 = nullptr;    // 2-bit text, built with the first per-k structures
    uint64_t* d_tbad = nullptr;     // bitmap of non-ACGT text positions
    bool ax_scan = true;            // tuning "ax_scan": read scans of k <= 128 use k_scan_ax
    uint32_t ax_mproof = 1;         // tuning "ax_mproof": m-mer absence proofs for the windows around a mismatch
                                    // (1: known and unknown mismatches, 2: known ones only, 0: off)
    uint32_t ax_load = 0;           // tuning "ax_load": anchor-table load factor, percent (0: default 35)
    uint32_t grid_blocks_ax = 65535;  // tuning "grid_blocks_ax"
    uint32_t blocks_per_cu_ax = 0;  // tuning "blocks_per_cu_ax" (0: as many as registers/LDS allow)
    uint32_t ax_generations = 1;    // tuning "ax_generations": grid = this many times the resident blocks (1: one
                                    // persistent generation; more: smaller pools, freed slots refilled by new blocks)
    std::mutex ax_mu;
    std::map<uint32_t, speq::AxTable> axtabs;
    std::mutex events_mu;  // launches may come from several host threads (pipelines, concurrent scans)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    double timed_ms = 0.0;
    uint64_t timed_launches = 0;
    // kernel of the last read scan (tuning key "last_kernel", read only): 0 LF steps (k_scan), 1 k-mer table
    // (k_scan, KT), 2 pipelined k-mer table (k_scan_kt), 3 anchor-and-extend (k_scan_ax)
    int last_kernel = -1;
};

namespace speq {
DevView search_view(const speq_device_index* d, uint32_t k);  // the FM view a search of k-mers uses (scan_kernels.hip)
AxTable build_ax(speq_device_index* d, uint32_t k);
const AxTable* ensure_ax(speq_device_index* d, uint32_t k);
uint32_t ax_effective_load(const speq_device_index* d);  // the anchor table's load factor (percent) builds use
bool launch_ax(speq_device_index* d, int mode, bool paired, const speq_dev::UnitSrc& src, hipStream_t st,
               unsigned long long* a, double* w);
}  // namespace speq
