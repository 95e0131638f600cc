// Internal entry points of the device half (scan_kernels.hip) used by the host-side streaming pipeline.
#pragma once
#include <cstdint>

#include "speq_scan.h"

namespace speq {
// Enqueues one k_scan launch over reads already in device memory on `stream`; counters accumulate into d_counts
// (and d_weights in local mode); em_mult/em_hi record multi-group intervals when non-null (EM scans).
void launch_reads_scan(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual, const uint64_t* d_offsets,
                       uint64_t n_reads, const speq_scan_params* p, uint64_t* d_counts, double* d_weights,
                       uint32_t* em_mult, uint32_t* em_hi, void* stream);
// Host-buffer scan through a pinned-slot pipeline (pipeline.cpp); counts/weights overwritten with the totals.
void scan_host_pipelined(speq_device_index* d, const uint8_t* seq, const uint8_t* qual, const uint64_t* offsets,
                         uint64_t n_reads, const speq_scan_params* p, speq_em* em, uint64_t* counts,
                         double* weights);
// Per-device cache of idle pipelines (pinned slots are costly to allocate): take one with >= n_slots slots
// (rebinding params/em) or create it; return it only after a successful speq_pipeline_finish (counters zero).
speq_pipeline* acquire_cached_pipeline(speq_device_index* d, const speq_scan_params* p, speq_em* em, uint64_t bytes,
                                       uint64_t records, uint32_t n_slots);
void return_cached_pipeline(speq_device_index* d, speq_pipeline* pl);
// Frees the idle host-scan pipelines cached for a device (called by speq_device_close).
void release_host_pipelines(const speq_device_index* d);
// GPU FASTQ parsing (fastq_gpu.hip): scratch bytes for a block pair, and the asynchronous parse into k_scan's layout.
size_t fastq_gpu_scratch_bytes(uint64_t raw_bytes, uint64_t records_per_file, bool paired);
void launch_fastq_parse(const uint8_t* d_raw, uint64_t len1, uint64_t len2, uint64_t n, bool paired, void* d_scratch,
                        size_t scratch_bytes, uint8_t* d_seq, uint8_t* d_qual, uint64_t* d_off, uint32_t* d_err,
                        uint64_t* d_total_bases, void* stream);
// Packed bases (one byte per base: bits 0-1 A C G T, bits 2-7 Phred clamped to [0, 41] or 63 for N) back to the
// ASCII (seq, qual) layout of the scan kernels (fastq_gpu.hip), and the host packer of that format (pipeline.cpp).
void launch_unpack_bases(const uint8_t* d_packed, uint64_t n, uint8_t* d_seq, uint8_t* d_qual, void* stream);
void pack_bases(uint8_t* out, const uint8_t* seq, const uint8_t* qual, uint64_t n);
// Submits an acquired slot whose base buffer holds n_records PACKED reads (offsets as usual): half the bytes of
// (seq, qual) cross PCIe, and the GPU unpacks them before the scan (pipeline.cpp).
void pipeline_submit_packed(speq_pipeline* pl, int32_t slot, uint64_t n_records);
// Global mode: 2-bit bases + one bad bit per base (not ACGTU, or Phred <= cutoff), 3 bits per base instead of 16
// (fastq_gpu.hip unpacks, pipeline.cpp packs; the slot's base buffer holds the code words, then the bad words).
void launch_unpack_bases3(const uint64_t* d_codes, const uint32_t* d_bad, uint64_t n, uint8_t* d_seq, uint8_t* d_qual,
                          void* stream);
void pack_bases3(uint64_t* codes, uint32_t* bad, const uint8_t* seq, const uint8_t* qual, uint64_t n, uint32_t cutoff);
// ORs n bases into the 3-bit streams at base offset `at` (the words they touch must start zeroed): record by record.
// wide: 32-byte loads may run up to 31 bytes past seq + n and qual + n (the caller's buffer continues there).
void pack_bases3_append(uint64_t* codes, uint32_t* bad, uint64_t at, const uint8_t* seq, const uint8_t* qual,
                        uint64_t n, uint32_t cutoff, bool wide = false);
inline uint64_t packed3_bytes(uint64_t n) { return (n + 31) / 32 * 12; }
void pipeline_submit_packed3(speq_pipeline* pl, int32_t slot, uint64_t n_records);
// Submits an acquired pipeline slot whose host buffer holds RAW four-line FASTQ text (file 1's block, then file
// 2's when paired, n records each): copied as is, parsed on the GPU, then scanned (pipeline.cpp).
// host1 / host2: copy the two blocks from these (pageable) host addresses instead of the slot's pinned buffer — the
// page-cache mapping of the file (SPEQ_FASTQ_DIRECT); the copy has left them when this returns (the runtime stages
// pageable sources before hipMemcpyAsync returns).
void pipeline_submit_raw(speq_pipeline* pl, int32_t slot, uint64_t len1, uint64_t len2, uint64_t n, bool paired,
                         const uint8_t* host1 = nullptr, const uint8_t* host2 = nullptr);
// Page-locks [p, p + n) of a read-only file mapping for direct DMA (hipHostRegister, read-only flag); false when the
// runtime refuses. host_unregister undoes it; pipeline_sync_copies waits for every H2D copy issued on pl so far.
bool host_register_readonly(void* p, size_t n);
void host_unregister(void* p);
void pipeline_sync_copies(speq_pipeline* pl);
// Acquires a slot for raw FASTQ text of up to `bytes` (no quality buffer; submit it with pipeline_submit_raw or
// release it with speq_pipeline_submit(pl, slot, 0)); *text receives the pinned host buffer.
int32_t pipeline_acquire_raw(speq_pipeline* pl, uint64_t bytes, uint8_t** text);
// Waits for every submitted batch and returns (and clears) the GPU parse error flags raised so far (0 = none).
uint32_t pipeline_take_parse_errors(speq_pipeline* pl);
// Bases parsed on the GPU by raw submits up to the last speq_pipeline_finish.
uint64_t pipeline_gpu_parsed_bases(const speq_pipeline* pl);
// Zeroes the interval histogram an EM scan has recorded so far (a stream restarted from its first record).
void em_clear(speq_em* em);
bool device_fastq_gpu(const speq_device_index* d);
uint32_t device_stream_lanes(const speq_device_index* d);
int device_ordinal(const speq_device_index* d);
// Code-object warm-up hooks, one per HIP translation unit (speq_device_warmup)
void warm_module_scan_kernels();
void warm_module_ax_scan();
void warm_module_build_gpu();
void warm_module_fastq_gpu();
// A non-blocking stream (hipStream_t) on `device` (the current device), from the pool speq_device_warmup filled, else a
// new one; bound to its hardware queue (a command has run on it). Its user destroys it with hipStreamDestroy.
void* pooled_stream(int device);
// Allocates n slot buffer sets of a FASTQ stream on `device` ahead of use (speq_stream_reserve): a fresh pipeline
// slot of at most (bytes, records) then takes one instead of allocating (pipeline.cpp).
void reserve_slot_buffers(int device, uint32_t n, uint64_t bytes, uint64_t records, bool paired);
// SPEQ_STARTUP_TRACE=1 (performance investigation only): "speq-trace: <what> <seconds>" on stderr, seconds since
// $SPEQ_T0 (ns since the epoch, set by a timing harness) or since the library was loaded
void startup_trace(const char* what);
uint32_t device_groups(const speq_device_index* d);
uint64_t device_text_len(const speq_device_index* d);  // FM text length n of the replica's index
}  // namespace speq
