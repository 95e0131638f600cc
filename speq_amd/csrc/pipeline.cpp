// Streaming scan pipeline: pinned host slots -> H2D on a copy stream -> k_scan on a compute stream.
//
// Replaces the reference's producer/consumer read path: one async_input_buffer thread parsing FASTQ for T-1 search
// workers (/root/reference/src/fm_scanner.cpp:138-141, :219-222; paired :651-655). Here producers fill page-locked
// slots; a submit enqueues three async copies on the copy stream, an event, and the kernel on the compute stream
// behind that event, so the PCIe copy of slot i+1 overlaps the scan of slot i. A slot is handed out again only after
// the event recorded behind its kernel has completed (its host and device buffers are then free).
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "capi_internal.hpp"
#include "em.hpp"
#include "scan_internal.hpp"

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw speq::DeviceError(std::string(what) + ": " + hipGetErrorString(e));
}

struct DevScope {
    int prev = -1;
    explicit DevScope(int dev) {
        hip_ok(hipGetDevice(&prev), "hipGetDevice");
        if (prev != dev) hip_ok(hipSetDevice(dev), "hipSetDevice");
    }
    ~DevScope() {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
    }
};

struct Slot {
    uint8_t* h_seq = nullptr;
    uint8_t* h_qual = nullptr;
    uint64_t* h_off = nullptr;
    uint8_t* d_seq = nullptr;
    uint8_t* d_qual = nullptr;
    uint64_t* d_off = nullptr;
    uint64_t cap_bytes = 0, cap_records = 0;
    hipEvent_t copied = nullptr, done = nullptr;
    bool pending = false;  // `done` recorded and not yet waited for
    // GPU FASTQ parsing (raw submits): parsed bases/qualities/offsets and scratch, allocated on first use
    uint8_t* d_pseq = nullptr;
    uint8_t* d_pqual = nullptr;
    uint64_t* d_poff = nullptr;
    void* d_scratch = nullptr;
    uint64_t parse_bytes = 0, parse_slots = 0;
    size_t scratch_bytes = 0;
};

// Pinned host memory of the slots: an aligned allocation, touched, then page-locked with hipHostRegister — 300 MB in
// 16 threads take 9-11 ms this way against 64-69 ms of hipHostMalloc (tools/upload_probe.cpp alloc,
// profiles/r06/cli/), and the copies from it run at the same DMA rate.
// Where registration is refused (a host whose page-locking limits differ from the GPU box's), hipHostMalloc;
// SPEQ_PINNED=hostmalloc takes that path always (tests).
std::mutex g_pinned_mu;
auto* g_host_malloced = new std::set<void*>();

void* pinned_alloc(size_t bytes) {
    const size_t n = (std::max<size_t>(bytes, 1) + 4095) & ~size_t(4095);
    const char* mode = std::getenv("SPEQ_PINNED");
    void* p = nullptr;
    if (!(mode && std::strcmp(mode, "hostmalloc") == 0)) {
        p = std::aligned_alloc(4096, n);
        if (!p) throw std::bad_alloc();
        std::memset(p, 0, n);
        if (hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess) return p;
        (void)hipGetLastError();
        std::free(p);
        p = nullptr;
    }
    hip_ok(hipHostMalloc(&p, n, hipHostMallocDefault), "hipHostMalloc");
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    g_host_malloced->insert(p);
    return p;
}

void pinned_free(void* p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        if (g_host_malloced->erase(p)) {
            (void)hipHostFree(p);
            return;
        }
    }
    (void)hipHostUnregister(p);
    std::free(p);
}

void free_parse(Slot& s) {
    if (s.d_pseq) (void)hipFree(s.d_pseq);
    if (s.d_pqual) (void)hipFree(s.d_pqual);
    if (s.d_poff) (void)hipFree(s.d_poff);
    if (s.d_scratch) (void)hipFree(s.d_scratch);
    s.d_pseq = s.d_pqual = nullptr;
    s.d_poff = nullptr;
    s.d_scratch = nullptr;
    s.parse_bytes = s.parse_slots = 0;
    s.scratch_bytes = 0;
}

void free_buffers(Slot& s) {
    pinned_free(s.h_seq);
    pinned_free(s.h_qual);
    pinned_free(s.h_off);
    if (s.d_seq) (void)hipFree(s.d_seq);
    if (s.d_qual) (void)hipFree(s.d_qual);
    if (s.d_off) (void)hipFree(s.d_off);
    s.h_seq = s.h_qual = s.d_seq = s.d_qual = nullptr;
    s.h_off = s.d_off = nullptr;
    s.cap_bytes = s.cap_records = 0;
}

// Slot buffer sets allocated ahead of a FASTQ stream (speq_stream_reserve, from the CLI's start-up thread while the
// index loads): pinned host text + offsets, device text + offsets, and the GPU parse buffers sized for the slot. At
// the start of a `speq scan` run the 16 parser threads' first slots allocated these on the critical path (up to 66 ms
// of pinned allocation per thread, profiles/r06/cli_trace_*).
struct PooledSlot {
    int device = 0;
    uint64_t bytes = 0, records = 0;
    uint8_t* h_seq = nullptr;
    uint64_t* h_off = nullptr;
    uint8_t* d_seq = nullptr;
    uint64_t* d_off = nullptr;
    uint8_t* d_pseq = nullptr;
    uint8_t* d_pqual = nullptr;
    uint64_t* d_poff = nullptr;
    void* d_scratch = nullptr;
    size_t scratch_bytes = 0;
};
std::mutex g_slot_mu;
auto* g_slot_pool = new std::vector<PooledSlot>();

// A fresh slot takes a pooled set of the current device with room for (bytes, records), if there is one.
bool take_pooled(Slot& s, uint64_t bytes, uint64_t records) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    PooledSlot e;
    {
        std::lock_guard<std::mutex> lk(g_slot_mu);
        auto it = std::find_if(g_slot_pool->begin(), g_slot_pool->end(), [&](const PooledSlot& x) {
            return x.device == dev && x.bytes >= bytes && x.records >= records;
        });
        if (it == g_slot_pool->end()) return false;
        e = *it;
        g_slot_pool->erase(it);
    }
    s.h_seq = e.h_seq;
    s.h_off = e.h_off;
    s.d_seq = e.d_seq;
    s.d_off = e.d_off;
    s.cap_bytes = e.bytes;
    s.cap_records = e.records;
    s.d_pseq = e.d_pseq;
    s.d_pqual = e.d_pqual;
    s.d_poff = e.d_poff;
    s.d_scratch = e.d_scratch;
    s.parse_bytes = e.bytes;
    s.parse_slots = e.records;
    s.scratch_bytes = e.scratch_bytes;
    return true;
}

// Grows the slot to at least (bytes, records); qualities (host + device) only when asked for or already there:
// raw-text submits (GPU FASTQ parsing) use the base buffer alone, which halves the pinned memory of a FASTQ stream.
void ensure_buffers(Slot& s, uint64_t bytes, uint64_t records, bool qual) {
    bytes = std::max<uint64_t>(bytes, 64);
    records = std::max<uint64_t>(records, 2);
    if (bytes > s.cap_bytes || records > s.cap_records) {
        bytes = std::max(bytes, s.cap_bytes);
        records = std::max(records, s.cap_records);
        qual = qual || s.h_qual;
        const bool fresh = s.cap_bytes == 0 && !s.d_pseq;
        free_buffers(s);
        if (!(fresh && take_pooled(s, bytes, records))) {
            s.h_seq = static_cast<uint8_t*>(pinned_alloc(bytes));
            s.h_off = static_cast<uint64_t*>(pinned_alloc((records + 1) * 8));
            hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_seq), bytes + 64), "hipMalloc");  // GPU parse: 16-B windows
            hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_off), (records + 1) * 8), "hipMalloc");
            s.cap_bytes = bytes;
            s.cap_records = records;
        }
    }
    if (qual && !s.h_qual) {
        s.h_qual = static_cast<uint8_t*>(pinned_alloc(s.cap_bytes));
        hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_qual), s.cap_bytes), "hipMalloc");
    }
}

}  // namespace

struct speq_pipeline {
    speq_device_index* d = nullptr;
    speq_scan_params p{};
    speq_em* em = nullptr;
    int device = 0;
    uint32_t G = 0;
    hipStream_t copy = nullptr, compute = nullptr;  // compute == lanes[0] (memsets and reads of the counters)
    std::vector<hipStream_t> lanes;                 // compute streams, used in turn by submits
    size_t next_lane = 0;                           // under submit_mu
    uint64_t* d_counts = nullptr;
    double* d_w = nullptr;
    std::vector<Slot> slots;    // buffers allocated on first acquire (ensure_buffers)
    uint64_t slot_bytes = 0, slot_records = 0;
    std::mutex mu;              // free list
    std::condition_variable cv;
    std::deque<int> free_slots;
    std::mutex submit_mu;       // stream order of copies and launches
    uint32_t* d_err = nullptr;  // GPU FASTQ parse errors (bit flags), checked by finish
    uint64_t* d_bases = nullptr;  // bases parsed on the GPU since the last finish
    uint64_t gpu_bases = 0;       // ... as of the last finish

    hipStream_t lane() { return lanes[next_lane++ % lanes.size()]; }
    void sync_lanes() {
        for (hipStream_t l : lanes) hip_ok(hipStreamSynchronize(l), "hipStreamSynchronize");
    }
    ~speq_pipeline() {
        for (hipStream_t l : lanes) (void)hipStreamSynchronize(l);
        if (copy) (void)hipStreamSynchronize(copy);
        if (d_err) (void)hipFree(d_err);
        if (d_bases) (void)hipFree(d_bases);
        for (Slot& s : slots) {
            free_buffers(s);
            free_parse(s);
            if (s.copied) (void)hipEventDestroy(s.copied);
            if (s.done) (void)hipEventDestroy(s.done);
        }
        if (d_counts) (void)hipFree(d_counts);
        if (d_w) (void)hipFree(d_w);
        if (copy) (void)hipStreamDestroy(copy);
        for (hipStream_t l : lanes) (void)hipStreamDestroy(l);
    }
};

extern "C" {

int speq_pipeline_create(speq_device_index* d, const speq_scan_params* params, speq_em* em, uint64_t slot_bytes,
                         uint64_t slot_records, uint32_t n_slots, speq_pipeline** out) {
    return speq::guarded([&] {
        if (!d || !params || !out) throw std::invalid_argument("speq_pipeline_create: null argument");
        if (n_slots < 2 || n_slots > 64) throw std::invalid_argument("speq_pipeline_create: n_slots must be in [2, 64]");
        if (params->paired && (slot_records & 1))
            throw std::invalid_argument("speq_pipeline_create: paired scans need an even slot_records");
        if (em && (em->dev != d || em->finalized))
            throw std::invalid_argument("speq_pipeline_create: EM histogram of another device, or finalized");
        if (params->mode != SPEQ_MODE_GLOBAL && params->mode != SPEQ_MODE_LOCAL)
            throw std::invalid_argument("speq_pipeline_create: bad mode");
        auto pl = std::make_unique<speq_pipeline>();
        pl->d = d;
        pl->p = *params;
        pl->em = em;
        pl->device = speq::device_ordinal(d);
        pl->G = speq::device_groups(d);
        DevScope g(pl->device);
        pl->copy = static_cast<hipStream_t>(speq::pooled_stream(pl->device));
        pl->lanes.resize(std::max<uint32_t>(1, speq::device_stream_lanes(d)), nullptr);
        for (hipStream_t& l : pl->lanes) l = static_cast<hipStream_t>(speq::pooled_stream(pl->device));
        pl->compute = pl->lanes[0];
        hip_ok(hipMalloc(reinterpret_cast<void**>(&pl->d_counts), SPEQ_COUNTS_LEN(pl->G) * 8), "hipMalloc");
        hip_ok(hipMemsetAsync(pl->d_counts, 0, SPEQ_COUNTS_LEN(pl->G) * 8, pl->compute), "hipMemset");
        hip_ok(hipMalloc(reinterpret_cast<void**>(&pl->d_err), 16), "hipMalloc");
        hip_ok(hipMemsetAsync(pl->d_err, 0, 16, pl->compute), "hipMemset");
        hip_ok(hipMalloc(reinterpret_cast<void**>(&pl->d_bases), 8), "hipMalloc");
        hip_ok(hipMemsetAsync(pl->d_bases, 0, 8, pl->compute), "hipMemset");
        hip_ok(hipMalloc(reinterpret_cast<void**>(&pl->d_w), std::max<uint32_t>(pl->G, 1) * 8), "hipMalloc");
        hip_ok(hipMemsetAsync(pl->d_w, 0, std::max<uint32_t>(pl->G, 1) * 8, pl->compute), "hipMemset");
        pl->slots.resize(n_slots);
        pl->slot_bytes = slot_bytes;
        pl->slot_records = slot_records;
        for (uint32_t i = 0; i < n_slots; ++i) {
            Slot& s = pl->slots[i];
            hip_ok(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming), "hipEventCreate");
            hip_ok(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate");
            pl->free_slots.push_back((int)i);
        }
        hip_ok(hipStreamSynchronize(pl->compute), "hipStreamSynchronize");
        *out = pl.release();
    });
}

}  // extern "C"

namespace {
// Next free slot (waits), its previous batch finished, buffers of at least (bytes, records) and qualities if asked.
int take_slot(speq_pipeline* pl, uint64_t bytes, uint64_t records, bool qual) {
    int i;
    {
        std::unique_lock<std::mutex> lk(pl->mu);
        pl->cv.wait(lk, [&] { return !pl->free_slots.empty(); });
        i = pl->free_slots.front();
        pl->free_slots.pop_front();
    }
    try {
        Slot& s = pl->slots[(size_t)i];
        if (s.pending) {
            hip_ok(hipEventSynchronize(s.done), "hipEventSynchronize");
            s.pending = false;
        }
        DevScope g(pl->device);
        ensure_buffers(s, bytes, records, qual);
    } catch (...) {
        {
            std::lock_guard<std::mutex> lk(pl->mu);
            pl->free_slots.push_back(i);
        }
        pl->cv.notify_one();
        throw;
    }
    return i;
}
}  // namespace

extern "C" {

int speq_pipeline_acquire(speq_pipeline* pl, speq_slot* out) {
    return speq::guarded([&] {
        if (!pl || !out) throw std::invalid_argument("speq_pipeline_acquire: null argument");
        const int i = take_slot(pl, pl->slot_bytes, pl->slot_records, true);
        Slot& s = pl->slots[(size_t)i];
        out->seq = s.h_seq;
        out->qual = s.h_qual;
        out->offsets = s.h_off;
        out->cap_bytes = s.cap_bytes;
        out->cap_records = s.cap_records;
        out->slot = i;
    });
}

int speq_pipeline_reserve(speq_pipeline* pl, speq_slot* slot, uint64_t bytes, uint64_t records) {
    return speq::guarded([&] {
        if (!pl || !slot || slot->slot < 0 || (size_t)slot->slot >= pl->slots.size())
            throw std::invalid_argument("speq_pipeline_reserve: bad slot");
        Slot& s = pl->slots[(size_t)slot->slot];
        if (bytes > s.cap_bytes || records > s.cap_records || !s.h_qual) {
            DevScope g(pl->device);
            ensure_buffers(s, bytes, records, true);
        }
        slot->seq = s.h_seq;
        slot->qual = s.h_qual;
        slot->offsets = s.h_off;
        slot->cap_bytes = s.cap_bytes;
        slot->cap_records = s.cap_records;
    });
}

int speq_pipeline_submit(speq_pipeline* pl, int32_t slot, uint64_t n_records) {
    auto release = [&] {
        {
            std::lock_guard<std::mutex> lk(pl->mu);
            pl->free_slots.push_back(slot);
        }
        pl->cv.notify_one();
    };
    if (!pl || slot < 0 || (size_t)slot >= pl->slots.size())
        return speq::guarded([] { throw std::invalid_argument("speq_pipeline_submit: bad slot"); });
    const int rc = speq::guarded([&] {
        Slot& s = pl->slots[(size_t)slot];
        if (n_records == 0) return;
        if (n_records > s.cap_records) throw std::invalid_argument("speq_pipeline_submit: more records than capacity");
        if (pl->p.paired && (n_records & 1))
            throw std::invalid_argument("speq_pipeline_submit: paired scan needs an even record count");
        const uint64_t* off = s.h_off;
        if (off[0] != 0) throw std::invalid_argument("speq_pipeline_submit: offsets[0] must be 0");
        for (uint64_t i = 0; i < n_records; ++i)
            if (off[i + 1] < off[i]) throw std::invalid_argument("speq_pipeline_submit: offsets must be non-decreasing");
        const uint64_t bytes = off[n_records];
        if (bytes > s.cap_bytes) throw std::invalid_argument("speq_pipeline_submit: offsets exceed the slot capacity");
        DevScope g(pl->device);
        std::lock_guard<std::mutex> lk(pl->submit_mu);
        if (bytes) {
            hip_ok(hipMemcpyAsync(s.d_seq, s.h_seq, bytes, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
            hip_ok(hipMemcpyAsync(s.d_qual, s.h_qual, bytes, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
        }
        hip_ok(hipMemcpyAsync(s.d_off, s.h_off, (n_records + 1) * 8, hipMemcpyHostToDevice, pl->copy),
               "hipMemcpyAsync");
        hip_ok(hipEventRecord(s.copied, pl->copy), "hipEventRecord");
        hipStream_t cs = pl->lane();
        hip_ok(hipStreamWaitEvent(cs, s.copied, 0), "hipStreamWaitEvent");
        speq::launch_reads_scan(pl->d, s.d_seq, s.d_qual, s.d_off, n_records, &pl->p, pl->d_counts, pl->d_w,
                                pl->em ? pl->em->d_mult : nullptr, pl->em ? pl->em->d_hi : nullptr, cs);
        hip_ok(hipEventRecord(s.done, cs), "hipEventRecord");
        s.pending = true;
    });
    release();
    return rc;
}

}  // extern "C"

namespace speq {
void pipeline_submit_raw(speq_pipeline* pl, int32_t slot, uint64_t len1, uint64_t len2, uint64_t n, bool paired,
                         const uint8_t* host1, const uint8_t* host2) {
    struct Release {
        speq_pipeline* pl;
        int32_t slot;
        ~Release() {
            {
                std::lock_guard<std::mutex> lk(pl->mu);
                pl->free_slots.push_back(slot);
            }
            pl->cv.notify_one();
        }
    } release{pl, slot};
    if (slot < 0 || (size_t)slot >= pl->slots.size()) throw std::invalid_argument("pipeline_submit_raw: bad slot");
    Slot& s = pl->slots[(size_t)slot];
    if (n == 0) return;
    if (len1 + len2 > s.cap_bytes) throw std::invalid_argument("pipeline_submit_raw: raw bytes exceed the slot");
    if ((bool)pl->p.paired != paired) throw std::invalid_argument("pipeline_submit_raw: paired mismatch");
    const uint64_t n_slots = paired ? 2 * n : n;
    DevScope g(pl->device);
    // parse buffers: bases <= raw bytes; the slot was acquired, so nothing in flight uses them
    const size_t need_scratch = fastq_gpu_scratch_bytes(std::max(len1, len2), n, paired);
    if (len1 + len2 > s.parse_bytes || n_slots > s.parse_slots || need_scratch > s.scratch_bytes) {
        // hipFree waits for the whole device, so size for the slot's capacity (and grow by half) to keep
        // reallocation out of the steady state
        const uint64_t pb = std::max({len1 + len2, s.parse_bytes * 3 / 2, s.cap_bytes});
        const uint64_t ps = std::max({n_slots, s.parse_slots * 3 / 2, s.cap_records});
        const size_t sb = std::max({need_scratch, s.scratch_bytes * 3 / 2,
                                    fastq_gpu_scratch_bytes(pb / (paired ? 2 : 1), ps / (paired ? 2 : 1), paired)});
        free_parse(s);
        hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_pseq), pb), "hipMalloc");
        hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_pqual), pb), "hipMalloc");
        hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_poff), (ps + 1) * 8), "hipMalloc");
        hip_ok(hipMalloc(&s.d_scratch, sb), "hipMalloc");
        s.parse_bytes = pb;
        s.parse_slots = ps;
        s.scratch_bytes = sb;
    }
    std::lock_guard<std::mutex> lk(pl->submit_mu);
    if (host1) {  // straight from the file's mapping (pageable: staged by the runtime, no slot copy on this thread)
        hip_ok(hipMemcpyAsync(s.d_seq, host1, len1, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
        if (len2) hip_ok(hipMemcpyAsync(s.d_seq + len1, host2, len2, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
    } else {
        hip_ok(hipMemcpyAsync(s.d_seq, s.h_seq, len1 + len2, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
    }
    hip_ok(hipEventRecord(s.copied, pl->copy), "hipEventRecord");
    hipStream_t cs = pl->lane();
    hip_ok(hipStreamWaitEvent(cs, s.copied, 0), "hipStreamWaitEvent");
    launch_fastq_parse(s.d_seq, len1, len2, n, paired, s.d_scratch, s.scratch_bytes, s.d_pseq, s.d_pqual, s.d_poff,
                       pl->d_err, pl->d_bases, cs);
    launch_reads_scan(pl->d, s.d_pseq, s.d_pqual, s.d_poff, n_slots, &pl->p, pl->d_counts, pl->d_w,
                      pl->em ? pl->em->d_mult : nullptr, pl->em ? pl->em->d_hi : nullptr, cs);
    hip_ok(hipEventRecord(s.done, cs), "hipEventRecord");
    s.pending = true;
}

bool host_register_readonly(void* p, size_t n) {
    return hipHostRegister(p, n, hipHostRegisterReadOnly) == hipSuccess;
}
void host_unregister(void* p) { (void)hipHostUnregister(p); }
void pipeline_sync_copies(speq_pipeline* pl) {
    DevScope g(pl->device);
    hip_ok(hipStreamSynchronize(pl->copy), "hipStreamSynchronize");
}

// Host packer of the one-byte-per-base format (launch_unpack_bases): dna5 (A C G T, U as T, any case; everything else
// N = 63) and phred42 (byte - 33 clamped to [0, 41]), as the kernels read them. AVX2 when the CPU has it.
namespace {
inline uint8_t pack_one(uint8_t sc, uint8_t qc) {
    const uint32_t x = sc | 0x20u;
    const bool ok = x == 'a' || x == 'c' || x == 'g' || x == 't' || x == 'u';
    if (!ok) return 63u << 2;
    const uint32_t code = ((x >> 1) ^ (x >> 2)) & 3u;
    const uint32_t q = qc < 33u ? 0u : std::min<uint32_t>(qc - 33u, 41u);
    return (uint8_t)(code | (q << 2));
}

__attribute__((target("avx2"))) void pack_avx2(uint8_t* out, const uint8_t* seq, const uint8_t* qual, uint64_t n) {
    // streaming stores into a 32-B aligned pinned slot (no read-for-ownership; SPEQ_NT_COPY=0 turns them off)
    static const bool nt = [] {
        const char* e = std::getenv("SPEQ_NT_COPY");
        return !(e && e[0] == '0');
    }();
    const bool stream = nt && (reinterpret_cast<uintptr_t>(out) & 31u) == 0;
    const __m256i lc = _mm256_set1_epi8(0x20), q33 = _mm256_set1_epi8(33), q41 = _mm256_set1_epi8(41);
    const __m256i A = _mm256_set1_epi8('a'), Cc = _mm256_set1_epi8('c'), Gg = _mm256_set1_epi8('g'),
                  Tt = _mm256_set1_epi8('t'), Uu = _mm256_set1_epi8('u'), three = _mm256_set1_epi8(3),
                  nval = _mm256_set1_epi8((char)(63 << 2));
    uint64_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i x = _mm256_or_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(seq + i)), lc);
        const __m256i ok = _mm256_or_si256(
            _mm256_or_si256(_mm256_cmpeq_epi8(x, A), _mm256_cmpeq_epi8(x, Cc)),
            _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(x, Gg), _mm256_cmpeq_epi8(x, Tt)),
                            _mm256_cmpeq_epi8(x, Uu)));
        // ((x >> 1) ^ (x >> 2)) & 3 per byte (16-bit shifts: the bits that cross bytes are masked off)
        const __m256i code = _mm256_and_si256(_mm256_xor_si256(_mm256_srli_epi16(x, 1), _mm256_srli_epi16(x, 2)), three);
        const __m256i q = _mm256_min_epu8(
            _mm256_subs_epu8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(qual + i)), q33), q41);
        const __m256i v = _mm256_or_si256(code, _mm256_slli_epi16(q, 2));  // q <= 41: q << 2 stays in its byte
        if (stream) _mm256_stream_si256(reinterpret_cast<__m256i*>(out + i), _mm256_blendv_epi8(nval, v, ok));
        else _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i), _mm256_blendv_epi8(nval, v, ok));
    }
    for (; i < n; ++i) out[i] = pack_one(seq[i], qual[i]);
    if (stream) _mm_sfence();
}
}  // namespace

namespace {
// 2-bit code (bits 0-1) and bad flag (bit 7 set) of one base for pack_bases3
inline void pack3_one(uint8_t sc, uint8_t qc, uint32_t cutoff, uint64_t& code, bool& bad) {
    const uint32_t x = sc | 0x20u;
    const bool ok = x == 'a' || x == 'c' || x == 'g' || x == 't' || x == 'u';
    const uint32_t q = qc < 33u ? 0u : std::min<uint32_t>(qc - 33u, 41u);
    code = ok ? (((x >> 1) ^ (x >> 2)) & 3u) : 0u;
    bad = !ok || q <= cutoff;
}

void pack3_scalar(uint64_t* codes, uint32_t* bad, const uint8_t* seq, const uint8_t* qual, uint64_t n,
                  uint32_t cutoff, uint64_t w0) {
    for (uint64_t w = w0; w * 32 < n; ++w) {
        uint64_t c = 0;
        uint32_t b = 0;
        for (uint32_t i = 0; i < 32; ++i) {
            const uint64_t j = w * 32 + i;
            uint64_t ci = 0;
            bool bi = true;
            if (j < n) pack3_one(seq[j], qual[j], cutoff, ci, bi);
            c |= ci << (2 * i);
            b |= (uint32_t)bi << i;
        }
        codes[w] = c;
        bad[w] = b;
    }
}

__attribute__((target("avx2,bmi2"))) void pack3_avx2(uint64_t* codes, uint32_t* bad, const uint8_t* seq,
                                                     const uint8_t* qual, uint64_t n, uint32_t cutoff) {
    const __m256i lc = _mm256_set1_epi8(0x20), q33 = _mm256_set1_epi8(33), q41 = _mm256_set1_epi8(41);
    const __m256i A = _mm256_set1_epi8('a'), Cc = _mm256_set1_epi8('c'), Gg = _mm256_set1_epi8('g'),
                  Tt = _mm256_set1_epi8('t'), Uu = _mm256_set1_epi8('u'), three = _mm256_set1_epi8(3);
    const __m256i cut = _mm256_set1_epi8((char)std::min<uint32_t>(cutoff, 41u));
    const bool all_bad = cutoff >= 41u;
    uint64_t w = 0;
    for (; (w + 1) * 32 <= n; ++w) {
        const uint64_t i = w * 32;
        const __m256i x = _mm256_or_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(seq + i)), lc);
        const __m256i ok = _mm256_or_si256(
            _mm256_or_si256(_mm256_cmpeq_epi8(x, A), _mm256_cmpeq_epi8(x, Cc)),
            _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(x, Gg), _mm256_cmpeq_epi8(x, Tt)),
                            _mm256_cmpeq_epi8(x, Uu)));
        const __m256i code = _mm256_and_si256(
            _mm256_and_si256(_mm256_xor_si256(_mm256_srli_epi16(x, 1), _mm256_srli_epi16(x, 2)), three), ok);
        const __m256i q = _mm256_min_epu8(
            _mm256_subs_epu8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(qual + i)), q33), q41);
        // good <=> ok and q > cutoff (unsigned: max(q, cut) != cut)
        const __m256i qgood = _mm256_xor_si256(_mm256_cmpeq_epi8(_mm256_max_epu8(q, cut), cut),
                                               _mm256_set1_epi8(-1));
        const uint32_t good = (uint32_t)_mm256_movemask_epi8(_mm256_and_si256(ok, qgood));
        alignas(32) uint64_t cb[4];
        _mm256_store_si256(reinterpret_cast<__m256i*>(cb), code);
        uint64_t c = 0;
        for (int t = 0; t < 4; ++t) c |= _pext_u64(cb[t], 0x0303030303030303ull) << (16 * t);
        codes[w] = c;
        bad[w] = all_bad ? ~0u : ~good;
    }
    pack3_scalar(codes, bad, seq, qual, n, cutoff, w);
}
}  // namespace

namespace {
// one chunk of up to 32 bases: 2-bit codes (bases past n zero) and bad bits (past n zero)
inline void pack3_chunk_scalar(const uint8_t* seq, const uint8_t* qual, uint32_t n, uint32_t cutoff, uint64_t& c,
                               uint32_t& b) {
    c = 0;
    b = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t ci = 0;
        bool bi = true;
        pack3_one(seq[i], qual[i], cutoff, ci, bi);
        c |= ci << (2 * i);
        b |= (uint32_t)bi << i;
    }
}

__attribute__((target("avx2,bmi2"))) void pack3_append_avx2(uint64_t* codes, uint32_t* bad, uint64_t at,
                                                            const uint8_t* seq, const uint8_t* qual, uint64_t n,
                                                            uint32_t cutoff, bool wide) {
    const __m256i lc = _mm256_set1_epi8(0x20), q33 = _mm256_set1_epi8(33), q41 = _mm256_set1_epi8(41);
    const __m256i A = _mm256_set1_epi8('a'), Cc = _mm256_set1_epi8('c'), Gg = _mm256_set1_epi8('g'),
                  Tt = _mm256_set1_epi8('t'), Uu = _mm256_set1_epi8('u'), three = _mm256_set1_epi8(3);
    const __m256i cut = _mm256_set1_epi8((char)std::min<uint32_t>(cutoff, 41u));
    const bool all_bad = cutoff >= 41u;
    for (uint64_t i = 0; i < n; i += 32) {
        const uint32_t m = (uint32_t)std::min<uint64_t>(32, n - i);
        uint64_t c;
        uint32_t b;
        if (m == 32 || wide) {  // wide: 32-byte loads past the tail stay inside the caller's buffer
            const __m256i x = _mm256_or_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(seq + i)), lc);
            const __m256i ok = _mm256_or_si256(
                _mm256_or_si256(_mm256_cmpeq_epi8(x, A), _mm256_cmpeq_epi8(x, Cc)),
                _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(x, Gg), _mm256_cmpeq_epi8(x, Tt)),
                                _mm256_cmpeq_epi8(x, Uu)));
            const __m256i code = _mm256_and_si256(
                _mm256_and_si256(_mm256_xor_si256(_mm256_srli_epi16(x, 1), _mm256_srli_epi16(x, 2)), three), ok);
            const __m256i q = _mm256_min_epu8(
                _mm256_subs_epu8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(qual + i)), q33), q41);
            const __m256i qgood = _mm256_xor_si256(_mm256_cmpeq_epi8(_mm256_max_epu8(q, cut), cut),
                                                   _mm256_set1_epi8(-1));
            const uint32_t good = (uint32_t)_mm256_movemask_epi8(_mm256_and_si256(ok, qgood));
            alignas(32) uint64_t cb[4];
            _mm256_store_si256(reinterpret_cast<__m256i*>(cb), code);
            c = 0;
            for (int t = 0; t < 4; ++t) c |= _pext_u64(cb[t], 0x0303030303030303ull) << (16 * t);
            b = all_bad ? ~0u : ~good;
            if (m < 32) {
                c &= (1ull << (2 * m)) - 1ull;
                b &= (1u << m) - 1u;
            }
        } else {  // the record's tail: no reads past its last byte
            pack3_chunk_scalar(seq + i, qual + i, m, cutoff, c, b);
        }
        const uint64_t o = at + i, w = o >> 5;
        const uint32_t sh = (uint32_t)(o & 31u);
        codes[w] |= c << (2 * sh);
        bad[w] |= b << sh;
        if (sh) {
            codes[w + 1] |= c >> (64 - 2 * sh);
            bad[w + 1] |= b >> (32 - sh);
        }
    }
}

void pack3_append_scalar(uint64_t* codes, uint32_t* bad, uint64_t at, const uint8_t* seq, const uint8_t* qual,
                         uint64_t n, uint32_t cutoff) {
    for (uint64_t i = 0; i < n; i += 32) {
        const uint32_t m = (uint32_t)std::min<uint64_t>(32, n - i);
        uint64_t c;
        uint32_t b;
        pack3_chunk_scalar(seq + i, qual + i, m, cutoff, c, b);
        const uint64_t o = at + i, w = o >> 5;
        const uint32_t sh = (uint32_t)(o & 31u);
        codes[w] |= c << (2 * sh);
        bad[w] |= b << sh;
        if (sh) {
            codes[w + 1] |= c >> (64 - 2 * sh);
            bad[w + 1] |= b >> (32 - sh);
        }
    }
}
}  // namespace

void pack_bases3_append(uint64_t* codes, uint32_t* bad, uint64_t at, const uint8_t* seq, const uint8_t* qual,
                        uint64_t n, uint32_t cutoff, bool wide) {
    static const bool fast = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi2");
    if (fast) pack3_append_avx2(codes, bad, at, seq, qual, n, cutoff, wide);
    else pack3_append_scalar(codes, bad, at, seq, qual, n, cutoff);
}

void pack_bases3(uint64_t* codes, uint32_t* bad, const uint8_t* seq, const uint8_t* qual, uint64_t n,
                 uint32_t cutoff) {
    static const bool fast = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi2");
    if (fast) pack3_avx2(codes, bad, seq, qual, n, cutoff);
    else pack3_scalar(codes, bad, seq, qual, n, cutoff, 0);
}

void pack_bases(uint8_t* out, const uint8_t* seq, const uint8_t* qual, uint64_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) {
        pack_avx2(out, seq, qual, n);
        return;
    }
    for (uint64_t i = 0; i < n; ++i) out[i] = pack_one(seq[i], qual[i]);
}

void pipeline_submit_packed_impl(speq_pipeline* pl, int32_t slot, uint64_t n_records, bool three);
void pipeline_submit_packed(speq_pipeline* pl, int32_t slot, uint64_t n_records) {
    pipeline_submit_packed_impl(pl, slot, n_records, false);
}
void pipeline_submit_packed3(speq_pipeline* pl, int32_t slot, uint64_t n_records) {
    pipeline_submit_packed_impl(pl, slot, n_records, true);
}
void pipeline_submit_packed_impl(speq_pipeline* pl, int32_t slot, uint64_t n_records, bool three) {
    struct Release {
        speq_pipeline* pl;
        int32_t slot;
        ~Release() {
            {
                std::lock_guard<std::mutex> lk(pl->mu);
                pl->free_slots.push_back(slot);
            }
            pl->cv.notify_one();
        }
    } release{pl, slot};
    if (slot < 0 || (size_t)slot >= pl->slots.size()) throw std::invalid_argument("pipeline_submit_packed: bad slot");
    Slot& s = pl->slots[(size_t)slot];
    if (n_records == 0) return;
    if (n_records > s.cap_records) throw std::invalid_argument("pipeline_submit_packed: more records than capacity");
    if (pl->p.paired && (n_records & 1))
        throw std::invalid_argument("pipeline_submit_packed: paired scan needs an even record count");
    const uint64_t bytes = s.h_off[n_records];  // bases
    const uint64_t wire = three ? packed3_bytes(bytes) : bytes;
    if (s.h_off[0] != 0 || wire > s.cap_bytes) throw std::invalid_argument("pipeline_submit_packed: bad offsets");
    DevScope g(pl->device);
    if (bytes > s.parse_bytes || n_records > s.parse_slots) {  // unpacked (seq, qual): the parse buffers
        const uint64_t pb = std::max({bytes, s.parse_bytes * 3 / 2, s.cap_bytes});
        const uint64_t ps = std::max({n_records, s.parse_slots * 3 / 2, s.cap_records});
        free_parse(s);
        hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_pseq), pb + 16), "hipMalloc");
        hip_ok(hipMalloc(reinterpret_cast<void**>(&s.d_pqual), pb + 16), "hipMalloc");
        s.parse_bytes = pb;
        s.parse_slots = ps;
    }
    std::lock_guard<std::mutex> lk(pl->submit_mu);
    if (bytes) hip_ok(hipMemcpyAsync(s.d_seq, s.h_seq, wire, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(s.d_off, s.h_off, (n_records + 1) * 8, hipMemcpyHostToDevice, pl->copy), "hipMemcpyAsync");
    hip_ok(hipEventRecord(s.copied, pl->copy), "hipEventRecord");
    hipStream_t cs = pl->lane();
    hip_ok(hipStreamWaitEvent(cs, s.copied, 0), "hipStreamWaitEvent");
    if (three) {
        const uint64_t nw = (bytes + 31) / 32;
        launch_unpack_bases3(reinterpret_cast<const uint64_t*>(s.d_seq),
                             reinterpret_cast<const uint32_t*>(s.d_seq + nw * 8), bytes, s.d_pseq, s.d_pqual, cs);
    } else {
        launch_unpack_bases(s.d_seq, bytes, s.d_pseq, s.d_pqual, cs);
    }
    launch_reads_scan(pl->d, s.d_pseq, s.d_pqual, s.d_off, n_records, &pl->p, pl->d_counts, pl->d_w,
                      pl->em ? pl->em->d_mult : nullptr, pl->em ? pl->em->d_hi : nullptr, cs);
    hip_ok(hipEventRecord(s.done, cs), "hipEventRecord");
    s.pending = true;
}

int32_t pipeline_acquire_raw(speq_pipeline* pl, uint64_t bytes, uint8_t** text) {
    const int i = take_slot(pl, std::max(bytes, pl->slot_bytes), pl->slot_records, false);
    *text = pl->slots[(size_t)i].h_seq;
    return i;
}

uint32_t pipeline_take_parse_errors(speq_pipeline* pl) {
    DevScope g(pl->device);
    std::lock_guard<std::mutex> lk(pl->submit_mu);
    pl->sync_lanes();
    uint32_t err = 0;
    hip_ok(hipMemcpy(&err, pl->d_err, 4, hipMemcpyDeviceToHost), "hipMemcpy");
    if (err) hip_ok(hipMemset(pl->d_err, 0, 4), "hipMemset");
    return err;
}

uint64_t pipeline_gpu_parsed_bases(const speq_pipeline* pl) { return pl->gpu_bases; }
}  // namespace speq

extern "C" {

int speq_pipeline_finish(speq_pipeline* pl, uint64_t* counts, double* weights) {
    return speq::guarded([&] {
        if (!pl || !counts) throw std::invalid_argument("speq_pipeline_finish: null argument");
        if (pl->p.mode == SPEQ_MODE_LOCAL && !weights)
            throw std::invalid_argument("speq_pipeline_finish: local mode needs weights");
        DevScope g(pl->device);
        std::lock_guard<std::mutex> lk(pl->submit_mu);
        pl->sync_lanes();  // every batch's kernels (any lane) before the counters are read
        const size_t nc = SPEQ_COUNTS_LEN(pl->G);
        hip_ok(hipMemcpyAsync(counts, pl->d_counts, nc * 8, hipMemcpyDeviceToHost, pl->compute), "hipMemcpyAsync");
        if (weights && pl->p.mode == SPEQ_MODE_LOCAL)
            hip_ok(hipMemcpyAsync(weights, pl->d_w, pl->G * 8, hipMemcpyDeviceToHost, pl->compute), "hipMemcpyAsync");
        hip_ok(hipMemsetAsync(pl->d_counts, 0, nc * 8, pl->compute), "hipMemsetAsync");
        if (pl->d_w) hip_ok(hipMemsetAsync(pl->d_w, 0, pl->G * 8, pl->compute), "hipMemsetAsync");
        uint32_t err = 0;
        uint64_t bases = 0;
        hip_ok(hipMemcpyAsync(&err, pl->d_err, 4, hipMemcpyDeviceToHost, pl->compute), "hipMemcpyAsync");
        hip_ok(hipMemsetAsync(pl->d_err, 0, 4, pl->compute), "hipMemsetAsync");
        hip_ok(hipMemcpyAsync(&bases, pl->d_bases, 8, hipMemcpyDeviceToHost, pl->compute), "hipMemcpyAsync");
        hip_ok(hipMemsetAsync(pl->d_bases, 0, 8, pl->compute), "hipMemsetAsync");
        hip_ok(hipStreamSynchronize(pl->compute), "hipStreamSynchronize");
        pl->gpu_bases = bases;
        if (err)
            throw speq::IoError(std::string("malformed FASTQ record (GPU parse:") + ((err & 1) ? " header not '@'" : "") +
                                ((err & 2) ? " separator not '+'" : "") +
                                ((err & 4) ? " sequence/quality length mismatch" : "") +
                                ((err & 8) ? " truncated record" : "") + ")");
    });
}

void speq_pipeline_free(speq_pipeline* pl) { delete pl; }

}  // extern "C"

// ---- host-buffer scans (speq_scan_reads / speq_em_scan_reads) over the pipeline ----
// Whole units are cut into batches of <= 16 MiB of bases; up to four filler threads copy batches into pinned slots
// (pageable -> pinned memcpy) and submit them, so the PCIe copy and the kernel of different batches overlap.
namespace {
// Streams created ahead of use (speq_device_warmup): hipStreamCreate takes 3-10 ms per stream at the start of a
// process (5 of them were 36 ms of a `speq scan` run on the critical path: profiles/r06/cli_trace_*).
std::mutex g_stream_mu;
auto* g_streams = new std::multimap<int, hipStream_t>();
void* g_stream_scratch[64] = {};  // per device: 8 B that a stream's binding command writes

hipStream_t new_bound_stream(int device) {
    hipStream_t st = nullptr;
    hip_ok(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    void* scratch = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        if (device >= 0 && device < 64) {
            if (!g_stream_scratch[device]) hip_ok(hipMalloc(&g_stream_scratch[device], 8), "hipMalloc");
            scratch = g_stream_scratch[device];
        }
    }
    // HIP binds a stream to its hardware queue at its first command: one now (see speq_pipeline_create)
    if (scratch) hip_ok(hipMemsetAsync(scratch, 0, 8, st), "hipMemset");
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
    return st;
}
}  // namespace

namespace speq {
void startup_trace(const char* what) {
    static const bool on = [] {
        const char* v = std::getenv("SPEQ_STARTUP_TRACE");
        return v && *v && *v != '0';
    }();
    if (!on) return;
    static const double t0 = [] {
        const char* v = std::getenv("SPEQ_T0");
        if (v && *v) return std::strtod(v, nullptr) * 1e-9;
        return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    }();
    const double now = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "speq-trace: %-34s %.4f s\n", what, now - t0);
}

void reserve_slot_buffers(int device, uint32_t n, uint64_t bytes, uint64_t records, bool paired) {
    bytes = std::max<uint64_t>(bytes, 64);
    records = std::max<uint64_t>(records, 2);
    const size_t sb = fastq_gpu_scratch_bytes(bytes / (paired ? 2 : 1), records / (paired ? 2 : 1), paired);
    std::vector<PooledSlot> got(n);
    std::vector<std::string> err(n);
    std::vector<std::thread> ts;
    for (uint32_t i = 0; i < n; ++i)  // (pinned allocation is page-locking: one thread per set)
        ts.emplace_back([&, i] {
            try {
                DevScope g(device);
                PooledSlot& e = got[i];
                e.device = device;
                e.bytes = bytes;
                e.records = records;
                e.scratch_bytes = sb;
                e.h_seq = static_cast<uint8_t*>(pinned_alloc(bytes));
                e.h_off = static_cast<uint64_t*>(pinned_alloc((records + 1) * 8));
                hip_ok(hipMalloc(reinterpret_cast<void**>(&e.d_seq), bytes + 64), "hipMalloc");
                hip_ok(hipMalloc(reinterpret_cast<void**>(&e.d_off), (records + 1) * 8), "hipMalloc");
                hip_ok(hipMalloc(reinterpret_cast<void**>(&e.d_pseq), bytes), "hipMalloc");
                hip_ok(hipMalloc(reinterpret_cast<void**>(&e.d_pqual), bytes), "hipMalloc");
                hip_ok(hipMalloc(reinterpret_cast<void**>(&e.d_poff), (records + 1) * 8), "hipMalloc");
                hip_ok(hipMalloc(&e.d_scratch, sb), "hipMalloc");
            } catch (const std::exception& x) {
                err[i] = x.what();
            }
        });
    for (auto& t : ts) t.join();
    startup_trace("slot buffers reserved");
    std::lock_guard<std::mutex> lk(g_slot_mu);
    for (uint32_t i = 0; i < n; ++i) {
        PooledSlot& e = got[i];
        if (err[i].empty()) {
            g_slot_pool->push_back(e);
            continue;
        }
        // (a set that failed part-way is released; the stream allocates its own slots as before)
        pinned_free(e.h_seq);
        pinned_free(e.h_off);
        for (void* q : {(void*)e.d_seq, (void*)e.d_off, (void*)e.d_pseq, (void*)e.d_pqual, (void*)e.d_poff, e.d_scratch})
            if (q) (void)hipFree(q);
    }
    for (const std::string& x : err)
        if (!x.empty()) throw DeviceError("speq_stream_reserve: " + x);
}

void* pooled_stream(int device) {
    {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        auto it = g_streams->find(device);
        if (it != g_streams->end()) {
            hipStream_t st = it->second;
            g_streams->erase(it);
            return st;
        }
    }
    return new_bound_stream(device);
}
}  // namespace speq

extern "C" int speq_device_warmup(int device, uint32_t streams) {
    return speq::guarded([&] {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
            throw speq::DeviceError("no GPU visible (the scan path has no CPU fallback)");
        if (device < 0 || device >= ndev) throw std::invalid_argument("speq_device_warmup: bad device ordinal");
        if (streams > 16) throw std::invalid_argument("speq_device_warmup: at most 16 streams");
        {
            DevScope g(device);
            speq::startup_trace("warm-up: runtime up");
            hip_ok(hipFree(nullptr), "hipFree");  // the device's context
            speq::startup_trace("warm-up: context");
        }
        // the scan's three code objects (3-10 ms each alone) and the streams (~8 ms each) on threads of their own
        std::vector<std::thread> ts;
        std::vector<std::string> err(5);
        auto run = [&](int i, void (*f)()) {
            ts.emplace_back([&, i, f] {
                try {
                    DevScope g(device);
                    f();
                    static const char* names[4] = {"warm-up: scan_kernels code", "warm-up: ax_scan code",
                                                   "warm-up: build_gpu code", "warm-up: fastq_gpu code"};
                    speq::startup_trace(names[i]);
                } catch (const std::exception& x) {
                    err[i] = x.what();
                }
            });
        };
        run(0, speq::warm_module_scan_kernels);
        run(1, speq::warm_module_ax_scan);
        run(3, speq::warm_module_fastq_gpu);  // (not the index builder's: a scan never runs it)
        ts.emplace_back([&] {
            try {
                DevScope g(device);
                for (uint32_t i = 0; i < streams; ++i) {
                    hipStream_t st = new_bound_stream(device);
                    std::lock_guard<std::mutex> lk(g_stream_mu);
                    g_streams->emplace(device, st);
                }
                speq::startup_trace("warm-up: streams");
            } catch (const std::exception& x) {
                err[4] = x.what();
            }
        });
        for (auto& t : ts) t.join();
        for (const std::string& x : err)
            if (!x.empty()) throw speq::DeviceError("speq_device_warmup: " + x);
    });
}

namespace {
// Idle host-scan pipelines per device (pinned allocation costs more than a typical scan); never destroyed at exit.
std::mutex g_cache_mu;
auto* g_cache = new std::multimap<const speq_device_index*, speq_pipeline*>();

speq_pipeline* take_pipeline(speq_device_index* d, const speq_scan_params* p, speq_em* em, uint64_t bytes,
                             uint64_t recs, uint32_t n_slots) {
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        auto r = g_cache->equal_range(d);
        for (auto it = r.first; it != r.second; ++it) {
            speq_pipeline* pl = it->second;
            if (pl->slots.size() < n_slots || pl->lanes.size() != speq::device_stream_lanes(d)) continue;
            g_cache->erase(it);
            pl->p = *p;
            pl->em = em;
            // grow allocated slots now, while nothing is in flight (a mid-stream hipFree stalls the device)
            pl->slot_bytes = std::max(pl->slot_bytes, bytes);
            pl->slot_records = std::max(pl->slot_records, recs + (recs & 1));
            DevScope g(pl->device);
            for (Slot& s : pl->slots)
                if (s.h_seq && (s.cap_bytes < bytes || s.cap_records < recs + (recs & 1)))
                    ensure_buffers(s, bytes, recs + (recs & 1), false);
            return pl;
        }
    }
    speq_pipeline* pl = nullptr;
    if (speq_pipeline_create(d, p, em, bytes, recs + (recs & 1), n_slots, &pl) != SPEQ_OK)
        throw speq::DeviceError(speq_last_error());
    return pl;
}

void put_pipeline(speq_device_index* d, speq_pipeline* pl) {
    pl->em = nullptr;
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_cache->emplace(d, pl);
}
}  // namespace

namespace speq {
speq_pipeline* acquire_cached_pipeline(speq_device_index* d, const speq_scan_params* p, speq_em* em, uint64_t bytes,
                                       uint64_t records, uint32_t n_slots) {
    return take_pipeline(d, p, em, bytes, records, n_slots);
}
void return_cached_pipeline(speq_device_index* d, speq_pipeline* pl) { put_pipeline(d, pl); }

void release_host_pipelines(const speq_device_index* d) {
    std::vector<speq_pipeline*> v;
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        auto r = g_cache->equal_range(d);
        for (auto it = r.first; it != r.second; ++it) v.push_back(it->second);
        g_cache->erase(d);
    }
    for (speq_pipeline* pl : v) delete pl;
}

void scan_host_pipelined(speq_device_index* d, const uint8_t* seq, const uint8_t* qual, const uint64_t* offsets,
                         uint64_t n_reads, const speq_scan_params* p, speq_em* em, uint64_t* counts,
                         double* weights) {
    if (!d || !p || !counts || (!offsets && n_reads)) throw std::invalid_argument("speq_scan_reads: null argument");
    if (p->mode == SPEQ_MODE_LOCAL && !weights) throw std::invalid_argument("speq_scan_reads: local mode needs weights");
    if (p->paired && (n_reads & 1)) throw std::invalid_argument("speq_scan_reads: paired scan needs an even record count");
    const uint32_t G = device_groups(d);
    std::fill(counts, counts + SPEQ_COUNTS_LEN(G), 0ull);
    if (weights) std::fill(weights, weights + G, 0.0);
    if (n_reads == 0) return;
    for (uint64_t i = 0; i < n_reads; ++i)
        if (offsets[i + 1] < offsets[i]) throw std::invalid_argument("speq_scan_reads: offsets must be non-decreasing");
    if (offsets[n_reads] > offsets[0] && (!seq || !qual)) throw std::invalid_argument("speq_scan_reads: null read buffer");
    // 16 MiB batches, four filler threads: 4-32 MiB x 4-8 fillers all land at 32-34 GB/s of host bytes on the box
    // (profiles/r01/ab_host_batches.txt); 4 MiB loses to per-batch overheads.
    auto env_u = [](const char* name, uint64_t dflt) {  // A/B knobs (scripts/host_path_probe.py)
        const char* v = std::getenv(name);
        return v && *v ? std::strtoull(v, nullptr, 10) : dflt;
    };
    const char* hp = std::getenv("SPEQ_HOST_PACK");
    const bool packed = !(hp && hp[0] == '0');
    // packed batches: 8 MiB of reads, 12 fillers, 12 slots (profiles/r02/host_probe*.jsonl: cfg 2 host arrays
    // 5.5 -> 3.3 ms against 16 MiB x 8 x 6); ASCII: 16 MiB x 4 x 6 (profiles/r01/ab_host_batches.txt)
    const uint64_t BATCH_BYTES = env_u("SPEQ_HOST_BATCH_MB", packed ? 8 : 16) << 20, BATCH_RECORDS = 1u << 16;
    const uint64_t step = p->paired ? 2 : 1;
    std::vector<std::pair<uint64_t, uint64_t>> batches;
    uint64_t max_bytes = 1, max_recs = step;
    for (uint64_t r0 = 0; r0 < n_reads;) {
        uint64_t r1 = r0 + step;
        while (r1 < n_reads && r1 - r0 < BATCH_RECORDS && offsets[r1 + step] - offsets[r0] <= BATCH_BYTES) r1 += step;
        batches.emplace_back(r0, r1);
        max_bytes = std::max(max_bytes, offsets[r1] - offsets[r0]);
        max_recs = std::max(max_recs, r1 - r0);
        r0 = r1;
    }
    // Reads cross PCIe packed (SPEQ_HOST_PACK=0: ASCII bases and qualities as given, for A/B): one byte per base
    // (pack_bases) in local mode, 3 bits per base (pack_bases3) in global mode; filler threads pack the batches
    // straight into the pinned slots.
    // global mode reads only "bad or not" of a quality: 3 bits per base (SPEQ_HOST_PACK=1: the byte format)
    const bool three = packed && p->mode == SPEQ_MODE_GLOBAL && !(hp && hp[0] == '1');
    const uint32_t fillers = (uint32_t)std::min<size_t>(env_u("SPEQ_HOST_FILLERS", packed ? 12 : 4), batches.size());
    const uint32_t n_slots =
        (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(2, env_u("SPEQ_HOST_SLOTS", packed ? 12 : 6)));
    std::unique_ptr<speq_pipeline, void (*)(speq_pipeline*)> guard(take_pipeline(d, p, em, max_bytes, max_recs,
                                                                                 n_slots),
                                                                   speq_pipeline_free);
    speq_pipeline* pl = guard.get();
    std::atomic<size_t> next{0};
    std::mutex err_mu;
    std::string err;
    auto fill = [&] {
        for (;;) {
            const size_t b = next++;
            if (b >= batches.size()) return;
            speq_slot s;
            if (speq_pipeline_acquire(pl, &s) != SPEQ_OK) {
                std::lock_guard<std::mutex> lk(err_mu);
                if (err.empty()) err = speq_last_error();
                return;
            }
            const uint64_t r0 = batches[b].first, r1 = batches[b].second, base = offsets[r0];
            const uint64_t nb = offsets[r1] - base;
            if ((nb > s.cap_bytes || r1 - r0 > s.cap_records) &&
                speq_pipeline_reserve(pl, &s, nb, r1 - r0) != SPEQ_OK) {
                std::lock_guard<std::mutex> lk(err_mu);
                if (err.empty()) err = speq_last_error();
                (void)speq_pipeline_submit(pl, s.slot, 0);
                return;
            }
            for (uint64_t i = r0; i <= r1; ++i) s.offsets[i - r0] = offsets[i] - base;
            if (packed) {
                try {
                    if (three) {
                        const uint64_t nw = (nb + 31) / 32;
                        if (nb)
                            pack_bases3(reinterpret_cast<uint64_t*>(s.seq), reinterpret_cast<uint32_t*>(s.seq + nw * 8),
                                        seq + base, qual + base, nb, p->phred_cutoff);
                        pipeline_submit_packed3(pl, s.slot, r1 - r0);
                        continue;
                    }
                    if (nb) pack_bases(s.seq, seq + base, qual + base, nb);
                    pipeline_submit_packed(pl, s.slot, r1 - r0);
                } catch (const std::exception& e) {
                    std::lock_guard<std::mutex> lk(err_mu);
                    if (err.empty()) err = e.what();
                    return;
                }
                continue;
            }
            if (nb) {
                std::memcpy(s.seq, seq + base, nb);
                std::memcpy(s.qual, qual + base, nb);
            }
            if (speq_pipeline_submit(pl, s.slot, r1 - r0) != SPEQ_OK) {
                std::lock_guard<std::mutex> lk(err_mu);
                if (err.empty()) err = speq_last_error();
                return;
            }
        }
    };
    std::vector<std::thread> ts;
    for (uint32_t i = 1; i < fillers; ++i) ts.emplace_back(fill);
    fill();
    for (auto& t : ts) t.join();
    if (speq_pipeline_finish(pl, counts, weights) != SPEQ_OK) throw DeviceError(speq_last_error());
    if (!err.empty()) throw DeviceError(err);
    put_pipeline(d, guard.release());  // counters are zero again after finish
}
}  // namespace speq
