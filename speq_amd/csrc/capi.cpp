// Host half of the C ABI (speq_scan.h): errors, index build/persistence, introspection.
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "capi_internal.hpp"

namespace speq {
namespace {
thread_local std::string g_last_error;
}
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace speq

extern "C" {

const char* speq_last_error(void) { return speq::g_last_error.c_str(); }

int speq_abi_version(void) { return SPEQ_ABI_VERSION; }

void speq_free(void* p) { std::free(p); }

int speq_index_build(const char* seq, const uint64_t* rec_offsets, uint32_t n_records, const int32_t* group_of_rec,
                     uint32_t n_group_entries, uint32_t n_groups, const speq_build_opts* opts, speq_index** out) {
    return speq::guarded([&] {
        if (!rec_offsets || !out || (!group_of_rec && n_group_entries) || (!seq && n_records && rec_offsets[n_records]))
            throw std::invalid_argument("speq_index_build: null argument");
        for (uint32_t r = 0; r < n_records; ++r)
            if (rec_offsets[r + 1] < rec_offsets[r]) throw std::invalid_argument("speq_index_build: offsets must be non-decreasing");
        int gpu = -1;
        if (opts && opts->gpu_build) {
            const int ndev = speq_device_count();
            if (ndev <= 0) throw speq::DeviceError("speq_index_build: gpu_build requested but no GPU is visible");
            if (opts->device < 0 || opts->device >= ndev) throw std::invalid_argument("speq_index_build: bad device ordinal");
            gpu = opts->device;
        }
        // label_table 2 = auto: the table pays off once the index outgrows L2 (n >= 4 M symbols; cfg 3 +3 %,
        // cfg 2 -4 %: profiles/r01/ab_occupancy.txt)
        bool lab = opts && opts->label_table == 1;
        if (opts && opts->label_table == 2) {
            uint64_t n = 1;
            for (uint32_t r = 0; r < n_records; ++r) n += 2 * (rec_offsets[r + 1] - rec_offsets[r] + 1);
            lab = n >= (4ull << 20);
        }
        // triple_steps 2 = auto: the 64 three-symbol planes (10.7 B per symbol) while they stay addressable with
        // 32-bit buffer offsets, i.e. below ~400 M symbols
        bool tri = opts && opts->triple_steps == 1;
        if (opts && opts->triple_steps == 2 && opts->pair_steps) {
            uint64_t n = 1;
            for (uint32_t r = 0; r < n_records; ++r) n += 2 * (rec_offsets[r + 1] - rec_offsets[r] + 1);
            tri = (n / speq::OCC_BLOCK + 1) * 64 * 16 < (uint64_t(1) << 32) - 4096;
        }
        auto idx = std::make_unique<speq_index>();
        speq::fm_build(idx->fm, seq, rec_offsets, n_records, group_of_rec, n_group_entries, n_groups,
                       opts ? opts->prefix_q : 0, opts ? opts->threads : 0, opts ? opts->pair_steps != 0 : false,
                       lab, gpu, tri);
        *out = idx.release();
    });
}

int speq_index_save(const speq_index* idx, const char* path, const void* user_header, uint64_t header_len) {
    return speq::guarded([&] {
        if (!idx || !path || (!user_header && header_len)) throw std::invalid_argument("speq_index_save: null argument");
        speq::fm_save(idx->fm, path, user_header, header_len);
    });
}

static void copy_header(const std::vector<uint8_t>& h, void** user_header, uint64_t* header_len) {
    if (header_len) *header_len = h.size();
    if (user_header) {
        void* p = std::malloc(h.empty() ? 1 : h.size());
        if (!p) throw std::bad_alloc();
        if (!h.empty()) std::memcpy(p, h.data(), h.size());
        *user_header = p;
    }
}

int speq_index_load(const char* path, speq_index** out, void** user_header, uint64_t* header_len) {
    return speq::guarded([&] {
        if (!path || !out) throw std::invalid_argument("speq_index_load: null argument");
        auto idx = std::make_unique<speq_index>();
        std::vector<uint8_t> h;
        speq::fm_load(idx->fm, path, &h);
        copy_header(h, user_header, header_len);
        *out = idx.release();
    });
}

int speq_index_read_header(const char* path, void** user_header, uint64_t* header_len) {
    return speq::guarded([&] {
        if (!path) throw std::invalid_argument("speq_index_read_header: null argument");
        std::vector<uint8_t> h;
        speq::fm_read_header(path, h);
        copy_header(h, user_header, header_len);
    });
}

void speq_index_free(speq_index* idx) { delete idx; }

int speq_index_get_info(const speq_index* idx, speq_index_info* info) {
    return speq::guarded([&] {
        if (!idx || !info) throw std::invalid_argument("speq_index_get_info: null argument");
        const speq::FmIndex& f = idx->fm;
        info->n = f.n;
        info->n_texts = f.n_texts;
        info->n_records = f.n_records;
        info->n_groups = f.n_groups;
        info->prefix_q = f.prefix_q;
        info->pair_steps = f.occ2.empty() ? 0u : 1u;
        info->label_table = f.lab.empty() ? 0u : 1u;
        info->triple_steps = f.occ3.empty() ? 0u : 1u;
        info->n_runs = f.run_label.size();
        info->device_bytes = f.device_bytes();
    });
}

int speq_index_array(const speq_index* idx, const char* name, const void** ptr, uint64_t* bytes) {
    return speq::guarded([&] {
        if (!idx || !name || !ptr || !bytes) throw std::invalid_argument("speq_index_array: null argument");
        const speq::FmIndex& f = idx->fm;
        const std::string n(name);
        auto set = [&](const void* p, uint64_t b) { *ptr = p; *bytes = b; };
        if (n == "text") set(f.text.data(), f.text.size());
        else if (n == "sa") set(f.sa.data(), f.sa.size() * 4);
        else if (n == "occ") set(f.occ.data(), f.occ.size() * sizeof(speq::OccEntry));
        else if (n == "occ2") set(f.occ2.data(), f.occ2.size() * sizeof(speq::OccEntry));
        else if (n == "occ3") set(f.occ3.data(), f.occ3.size() * sizeof(speq::OccEntry));
        else if (n == "lab") set(f.lab.data(), f.lab.size() * 4);
        else if (n == "runs") set(f.runs.data(), f.runs.size() * sizeof(speq::OccEntry));
        else if (n == "run_label") set(f.run_label.data(), f.run_label.size() * 2);
        else if (n == "prefix") set(f.prefix.data(), f.prefix.size() * 4);
        else if (n == "prefix_q1") set(f.prefix1.data(), f.prefix1.size() * 4);
        else if (n == "prefix_q2") set(f.prefix2.data(), f.prefix2.size() * 4);
        else if (n == "C") set(f.C, sizeof(f.C));
        else if (n == "text_start") set(f.text_start.data(), f.text_start.size() * 8);
        else if (n == "text_group") set(f.text_group.data(), f.text_group.size() * 4);
        else throw std::invalid_argument("speq_index_array: unknown array " + n);
    });
}

}  // extern "C"
