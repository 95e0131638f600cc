// FM-index builder and persistence. See fm_index.hpp for the layout.
//
// Reference behaviour followed:
//   texts [fwd_r, revcomp(fwd_r)] per record, in FASTA order   /root/reference/src/fm_indexer.cpp:25-33
//   text -> group: group_scaffolds[t / 2]                       /root/reference/src/fm_scanner.cpp:74-77
#include "fm_index.hpp"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <stdexcept>
#include <thread>

#include "sais.hpp"
#include "speq_errors.hpp"

namespace speq {
namespace {

void parallel_for(uint64_t n, uint32_t threads, const std::function<void(uint64_t, uint64_t)>& body) {
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    threads = (uint32_t)std::min<uint64_t>(threads, std::max<uint64_t>(1, n / 65536));
    if (threads <= 1) { body(0, n); return; }
    std::vector<std::thread> pool;
    uint64_t chunk = (n + threads - 1) / threads;
    for (uint32_t t = 0; t < threads; ++t) {
        uint64_t b = t * chunk, e = std::min(n, b + chunk);
        if (b >= e) break;
        pool.emplace_back(body, b, e);
    }
    for (auto& th : pool) th.join();
}

inline uint32_t popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }

inline uint32_t entry_rank(const OccEntry& e, uint32_t r) {  // count + #set bits among the first r (0..96)
    uint32_t c = e.count;
    for (uint32_t w = 0; w < 3; ++w) {
        uint32_t lo = w * 32;
        if (r >= lo + 32) c += popc32(e.bits[w]);
        else if (r > lo) c += popc32(e.bits[w] & ((1u << (r - lo)) - 1u));
    }
    return c;
}

// Fills entries (stride `stride`, starting at entries[0]) from a per-position predicate.
template <typename Pred>
void fill_bitvector(OccEntry* entries, size_t stride, uint64_t n, uint64_t n_blocks, Pred pred, uint32_t threads) {
    // pass 1: per-block popcounts (parallel), pass 2: prefix sums (serial)
    std::vector<uint32_t> block_pop(n_blocks, 0);
    parallel_for(n_blocks, threads, [&](uint64_t b0, uint64_t b1) {
        for (uint64_t b = b0; b < b1; ++b) {
            OccEntry& e = entries[b * stride];
            e.bits[0] = e.bits[1] = e.bits[2] = 0;
            uint32_t pop = 0;
            for (uint32_t r = 0; r < OCC_BLOCK; ++r) {
                uint64_t i = b * OCC_BLOCK + r;
                if (i >= n) break;
                if (pred(i)) { e.bits[r >> 5] |= 1u << (r & 31); ++pop; }
            }
            block_pop[b] = pop;
        }
    });
    uint64_t acc = 0;
    for (uint64_t b = 0; b < n_blocks; ++b) {
        if (acc > 0xFFFFFFFFull) throw std::runtime_error("fm_build: rank overflows 32 bits");
        entries[b * stride].count = (uint32_t)acc;
        acc += block_pop[b];
    }
}

}  // namespace

uint64_t FmIndex::device_bytes() const {
    return occ.size() * sizeof(OccEntry) + occ2.size() * sizeof(OccEntry) + occ3.size() * sizeof(OccEntry) +
           runs.size() * sizeof(OccEntry) +
           run_label.size() * 2 + lab.size() * 4 + (prefix.size() + prefix1.size() + prefix2.size()) * 4 + text.size() + text_start.size() * 8 + text_group.size() * 4;
}

uint32_t FmIndex::lf(uint8_t sym, uint64_t i) const {
    uint64_t b = i / OCC_BLOCK;
    uint32_t r = (uint32_t)(i - b * OCC_BLOCK);
    const OccEntry& e = occ[(uint64_t)(sym - SYM_A) * n_blocks() + b];
    return entry_rank(e, r);
}

uint32_t FmIndex::rank(uint8_t sym, uint64_t i) const { return lf(sym, i) - C[sym]; }

uint32_t FmIndex::lf2(uint8_t a, uint8_t b, uint64_t i) const {
    uint64_t blk = i / OCC_BLOCK;
    uint32_t r = (uint32_t)(i - blk * OCC_BLOCK);
    return entry_rank(occ2[(uint64_t)((a - SYM_A) * 4 + (b - SYM_A)) * n_blocks() + blk], r);
}

uint32_t FmIndex::lf3(uint8_t a, uint8_t b, uint8_t c, uint64_t i) const {
    uint64_t blk = i / OCC_BLOCK;
    uint32_t r = (uint32_t)(i - blk * OCC_BLOCK);
    return entry_rank(occ3[(uint64_t)((a - SYM_A) * 16 + (b - SYM_A) * 4 + (c - SYM_A)) * n_blocks() + blk], r);
}

void triple_bases(const FmIndex& idx, uint32_t out[64]) {
    // #suffixes < "abc" = #p: T[p] < a, or T[p] = a and T[p+1] < b, or T[p..p+1] = ab and T[p+2] < c
    const uint8_t* T = idx.text.data();
    const uint64_t n = idx.n;
    std::vector<uint64_t> pc(SYM_COUNT * SYM_COUNT, 0), tc(SYM_COUNT * SYM_COUNT * SYM_COUNT, 0);
    for (uint64_t p = 0; p + 1 < n; ++p) {
        pc[T[p] * SYM_COUNT + T[p + 1]]++;
        if (p + 2 < n) tc[(T[p] * SYM_COUNT + T[p + 1]) * SYM_COUNT + T[p + 2]]++;
    }
    for (uint8_t a = SYM_A; a <= SYM_T; ++a)
        for (uint8_t b = SYM_A; b <= SYM_T; ++b)
            for (uint8_t c = SYM_A; c <= SYM_T; ++c) {
                uint64_t v = idx.C[a];
                for (uint8_t x = 0; x < b; ++x) v += pc[a * SYM_COUNT + x];
                for (uint8_t x = 0; x < c; ++x) v += tc[(a * SYM_COUNT + b) * SYM_COUNT + x];
                if (v > 0xFFFFFFFFull) throw std::runtime_error("fm_build: LF3 overflows 32 bits");
                out[(a - SYM_A) * 16 + (b - SYM_A) * 4 + (c - SYM_A)] = (uint32_t)v;
            }
}

uint64_t FmIndex::run_end(uint64_t i) const {
    // first j > i with B[j] = 1 (a label boundary), scanning the run bitvector entry by entry
    for (uint64_t j = i + 1; j < n;) {
        const uint64_t b = j / OCC_BLOCK;
        const uint32_t r = (uint32_t)(j - b * OCC_BLOCK);
        const OccEntry& e = runs[b];
        for (uint32_t w = r / 32; w < 3; ++w) {
            uint32_t bits = e.bits[w];
            if (w == r / 32) bits &= ~0u << (r % 32);
            if (bits) return std::min<uint64_t>(n, b * OCC_BLOCK + w * 32 + (uint64_t)__builtin_ctz(bits));
        }
        j = (b + 1) * OCC_BLOCK;
    }
    return n;
}

uint32_t FmIndex::run_of(uint64_t i) const {
    uint64_t b = i / OCC_BLOCK;
    uint32_t r = (uint32_t)(i - b * OCC_BLOCK);
    return entry_rank(runs[b], r + 1);
}

namespace {

template <typename Phase>
void build_arrays_host(FmIndex& idx, uint32_t threads, bool pair_steps, bool triple_steps, bool label_table,
                       Phase&& phase) {
    const uint64_t n = idx.n;
    // Suffix array
    idx.sa.resize(n);
    sais_u8(idx.text.data(), idx.sa.data(), (int64_t)n, SYM_COUNT);
    phase("sa");

    const uint64_t nb = idx.n_blocks();
    const uint8_t* T = idx.text.data();
    const int32_t* SA = idx.sa.data();
    auto bwt = [&](uint64_t i) -> uint8_t { return SA[i] == 0 ? (uint8_t)SYM_TERM : T[SA[i] - 1]; };

    idx.occ.assign(nb * 5, OccEntry{});
    for (uint8_t s = SYM_A; s <= SYM_N; ++s) {
        OccEntry* plane = idx.occ.data() + (uint64_t)(s - SYM_A) * nb;
        fill_bitvector(plane, 1, n, nb, [&](uint64_t i) { return bwt(i) == s; }, threads);
        // Fold C[s] into the block counts: an LF step is then entry.count + popcount, with no C[] lookup.
        for (uint64_t b = 0; b < nb; ++b) {
            if ((uint64_t)plane[b].count + idx.C[s] > 0xFFFFFFFFull) throw std::runtime_error("fm_build: LF overflows 32 bits");
            plane[b].count += idx.C[s];
        }
    }

    phase("occ");
    if (pair_steps) {
        // C2[ab] = #suffixes < "ab" = #positions p with T[p] < a, or T[p] == a and T[p+1] < b.
        uint64_t pc[SYM_COUNT][SYM_COUNT] = {{0}};
        for (uint64_t p = 0; p + 1 < n; ++p) pc[T[p]][T[p + 1]]++;
        idx.occ2.assign(nb * 16, OccEntry{});
        for (uint8_t a = SYM_A; a <= SYM_T; ++a) {
            for (uint8_t b = SYM_A; b <= SYM_T; ++b) {
                uint64_t c2 = idx.C[a];
                for (uint8_t c = 0; c < b; ++c) c2 += pc[a][c];
                OccEntry* plane = idx.occ2.data() + (uint64_t)((a - SYM_A) * 4 + (b - SYM_A)) * nb;
                fill_bitvector(plane, 1, n, nb, [&](uint64_t i) {
                    return SA[i] >= 2 && T[SA[i] - 2] == a && T[SA[i] - 1] == b;
                }, threads);
                for (uint64_t blk = 0; blk < nb; ++blk) {
                    if ((uint64_t)plane[blk].count + c2 > 0xFFFFFFFFull) throw std::runtime_error("fm_build: LF2 overflows");
                    plane[blk].count += (uint32_t)c2;
                }
            }
        }
    }

    phase("occ2");
    if (triple_steps) {
        // three symbols before each suffix as one code (0xFF when any is not in A..T or missing)
        std::vector<uint8_t> code(n);
        parallel_for(n, threads, [&](uint64_t i0, uint64_t i1) {
            for (uint64_t i = i0; i < i1; ++i) {
                const int64_t s = SA[i];
                uint8_t c = 0xFF;
                if (s >= 3) {
                    const uint8_t x = T[s - 3], y = T[s - 2], z = T[s - 1];
                    if (x >= SYM_A && x <= SYM_T && y >= SYM_A && y <= SYM_T && z >= SYM_A && z <= SYM_T)
                        c = (uint8_t)((x - SYM_A) * 16 + (y - SYM_A) * 4 + (z - SYM_A));
                }
                code[i] = c;
            }
        });
        uint32_t base[64];
        triple_bases(idx, base);
        idx.occ3.assign(nb * 64, OccEntry{});
        for (uint32_t pl = 0; pl < 64; ++pl) {
            OccEntry* plane = idx.occ3.data() + (uint64_t)pl * nb;
            fill_bitvector(plane, 1, n, nb, [&](uint64_t i) { return code[i] == pl; }, threads);
            for (uint64_t blk = 0; blk < nb; ++blk) {
                if ((uint64_t)plane[blk].count + base[pl] > 0xFFFFFFFFull) throw std::runtime_error("fm_build: LF3 overflows");
                plane[blk].count += base[pl];
            }
        }
    }
    phase("occ3");
    // Label of every SA position: group of the text that holds the suffix start.
    std::vector<uint16_t> label(n);
    const uint64_t* ts = idx.text_start.data();
    const uint32_t nt = idx.n_texts;
    parallel_for(n, threads, [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; ++i) {
            uint64_t pos = (uint64_t)SA[i];
            uint32_t t = (uint32_t)(std::upper_bound(ts, ts + nt + 1, pos) - ts) - 1;
            if (t >= nt) t = nt - 1;  // terminator
            label[i] = (uint16_t)idx.text_group[t];
        }
    });
    idx.runs.assign(nb, OccEntry{});
    fill_bitvector(idx.runs.data(), 1, n, nb, [&](uint64_t i) { return i > 0 && label[i] != label[i - 1]; }, threads);
    idx.run_label.clear();
    idx.run_label.push_back(label[0]);
    for (uint64_t i = 1; i < n; ++i)
        if (label[i] != label[i - 1]) idx.run_label.push_back(label[i]);
    if (label_table) {
        idx.lab.resize(n);
        uint64_t run_end = n;
        for (uint64_t i = n; i-- > 0;) {
            if (i + 1 < n && label[i] != label[i + 1]) run_end = i + 1;
            const uint64_t rem = std::min<uint64_t>(run_end - i, 0xFFFF);
            idx.lab[i] = (uint32_t)label[i] | ((uint32_t)rem << 16);
        }
    }

}

}  // namespace

void fm_build(FmIndex& idx, const char* seq, const uint64_t* rec_offsets, uint32_t n_records,
              const int32_t* group_of_rec, uint32_t n_group_entries, uint32_t n_groups, uint32_t prefix_q,
              uint32_t threads, bool pair_steps, bool label_table, int gpu_device, bool triple_steps) {
    if (n_records == 0) throw std::invalid_argument("fm_build: no reference records");
    if (n_groups == 0 || n_groups > 65535) throw std::invalid_argument("fm_build: n_groups must be in [1, 65535]");
    if (prefix_q > MAX_PREFIX_Q) throw std::invalid_argument("fm_build: prefix_q > 13");
    if (triple_steps && !pair_steps) throw std::invalid_argument("fm_build: triple steps need the pair planes");
    // Every record must belong to a group: the reference indexes group_scaffolds[t/2] unchecked
    // (fm_scanner.cpp:170, :1102, :1518) -- unassigned (-1) or missing entries are UB there, rejected here.
    if (n_group_entries < n_records)
        throw GroupsError("groupings assign " + std::to_string(n_group_entries) + " record indices but the reference has " +
                          std::to_string(n_records) + " records");
    for (uint32_t r = 0; r < n_records; ++r) {
        if (group_of_rec[r] < 0 || (uint32_t)group_of_rec[r] >= n_groups)
            throw GroupsError("reference record " + std::to_string(r) + " is not assigned to a group");
    }

    idx = FmIndex();
    idx.n_records = n_records;
    idx.n_texts = 2 * n_records;
    idx.n_groups = n_groups;
    idx.prefix_q = prefix_q;
    idx.group_of_rec.assign(group_of_rec, group_of_rec + n_group_entries);

    uint64_t total = 1;
    for (uint32_t r = 0; r < n_records; ++r) total += 2 * (rec_offsets[r + 1] - rec_offsets[r] + 1);
    if (total >= (uint64_t(1) << 31)) throw std::invalid_argument("fm_build: collection exceeds 2^31 symbols");
    idx.n = total;
    // the kernel addresses planes with 32-bit buffer offsets
    if (pair_steps && (total / OCC_BLOCK + 1) * 16 * sizeof(OccEntry) >= (uint64_t(1) << 32) - 4096)
        throw std::invalid_argument("fm_build: two-symbol planes exceed 4 GiB; build without pair steps");
    if (triple_steps && (total / OCC_BLOCK + 1) * 64 * sizeof(OccEntry) >= (uint64_t(1) << 32) - 4096)
        throw std::invalid_argument("fm_build: three-symbol planes exceed 4 GiB; build without triple steps");
    idx.text.resize(total);
    idx.text_start.resize(idx.n_texts + 1);
    idx.text_group.resize(idx.n_texts);
    uint64_t p = 0;
    for (uint32_t r = 0; r < n_records; ++r) {
        uint64_t b = rec_offsets[r], e = rec_offsets[r + 1], len = e - b;
        idx.text_start[2 * r] = p;
        for (uint64_t i = 0; i < len; ++i) idx.text[p + i] = ascii_to_sym((unsigned char)seq[b + i]);
        idx.text[p + len] = SYM_SEP;
        uint64_t q = p + len + 1;
        idx.text_start[2 * r + 1] = q;
        for (uint64_t i = 0; i < len; ++i) idx.text[q + i] = complement_sym(idx.text[p + len - 1 - i]);
        idx.text[q + len] = SYM_SEP;
        p = q + len + 1;
        idx.text_group[2 * r] = idx.text_group[2 * r + 1] = group_of_rec[r];
    }
    idx.text[p] = SYM_TERM;
    idx.text_start[idx.n_texts] = p;  // == n - 1
    const uint64_t n = idx.n;

    // C array
    uint64_t cnt[SYM_COUNT] = {0};
    for (uint64_t i = 0; i < n; ++i) cnt[idx.text[i]]++;
    idx.C[0] = 0;
    for (int c = 0; c < SYM_COUNT; ++c) idx.C[c + 1] = idx.C[c] + (uint32_t)cnt[c];

    const bool show = std::getenv("SPEQ_BUILD_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!show) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "fm_build: %-10s %.3f s\n", what, std::chrono::duration<double>(t - t_last).count());
        t_last = t;
    };
    phase("text");

    if (gpu_device >= 0) {
        fm_build_arrays_gpu(idx, gpu_device, pair_steps, triple_steps, label_table, show);
    } else {
        build_arrays_host(idx, threads, pair_steps, triple_steps, label_table, phase);
    }
    phase("labels");
    // q-mer interval table, built level by level by backward extension.
    if (prefix_q > 0) {
        const uint64_t Q = uint64_t(1) << (2 * prefix_q);
        std::vector<uint32_t> cur(2 * 4), next;
        for (uint32_t c = 0; c < 4; ++c) {
            cur[2 * c] = idx.C[SYM_A + c];
            cur[2 * c + 1] = idx.C[SYM_A + c + 1];
        }
        for (uint32_t len = 1; len < prefix_q; ++len) {
            if (len + 2 == prefix_q) idx.prefix2 = cur;
            if (len + 1 == prefix_q) idx.prefix1 = cur;
            uint64_t m = uint64_t(1) << (2 * len);  // number of len-mers
            next.assign(2 * m * 4, 0);
            // new (len+1)-mer = c . y ; code = c * 4^len + code(y)
            parallel_for(m * 4, threads, [&](uint64_t j0, uint64_t j1) {
                for (uint64_t j = j0; j < j1; ++j) {
                    uint32_t c = (uint32_t)(j / m);
                    uint64_t y = j % m;
                    uint32_t lo = cur[2 * y], hi = cur[2 * y + 1];
                    uint8_t s = (uint8_t)(SYM_A + c);
                    if (lo < hi) {
                        lo = idx.lf(s, lo);
                        hi = idx.lf(s, hi);
                    } else {
                        lo = hi = 0;
                    }
                    next[2 * j] = lo;
                    next[2 * j + 1] = hi;
                }
            });
            cur.swap(next);
        }
        if (cur.size() != 2 * Q) throw std::runtime_error("fm_build: prefix table size mismatch");
        idx.prefix.swap(cur);
    }
    phase("prefix");
}

// ---------------------------------------------------------------------------------------------
// Persistence: "SPEQIDX1" | u32 version | u32 0 | u64 header_len | header | fields | arrays
namespace {
constexpr char MAGIC[8] = {'S', 'P', 'E', 'Q', 'I', 'D', 'X', '1'};  // + FILE_VERSION
constexpr uint32_t FILE_VERSION = 7;

template <typename T>
void put(std::ofstream& os, const T& v) { os.write(reinterpret_cast<const char*>(&v), sizeof(T)); }
template <typename T>
void put_vec(std::ofstream& os, const std::vector<T>& v) {
    uint64_t count = v.size();
    put(os, count);
    if (count) os.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(count * sizeof(T)));
}
template <typename T>
void get(std::ifstream& is, T& v) {
    is.read(reinterpret_cast<char*>(&v), sizeof(T));
    if (!is) throw IoError("truncated index file");
}
template <typename T>
void get_vec(std::ifstream& is, std::vector<T>& v, uint64_t max_count) {
    uint64_t count = 0;
    get(is, count);
    if (count > max_count) throw IoError("corrupt index file (array too large)");
    v.resize(count);
    if (count) is.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(count * sizeof(T)));
    if (!is) throw IoError("truncated index file");
}

void read_preamble(std::ifstream& is, const std::string& path, std::vector<uint8_t>* header) {
    char magic[8];
    is.read(magic, 8);
    if (!is || std::memcmp(magic, MAGIC, 8) != 0) throw IoError("not a speq index file: " + path);
    uint32_t version = 0, zero = 0;
    get(is, version);
    get(is, zero);
    if (version != FILE_VERSION) throw IoError("unsupported index file version in " + path);
    uint64_t hl = 0;
    get(is, hl);
    if (hl > (uint64_t(1) << 32)) throw IoError("corrupt index header in " + path);
    std::vector<uint8_t> h(hl);
    if (hl) is.read(reinterpret_cast<char*>(h.data()), (std::streamsize)hl);
    if (!is) throw IoError("truncated index file " + path);
    if (header) header->swap(h);
}
}  // namespace

void fm_save(const FmIndex& idx, const std::string& path, const void* header, uint64_t header_len) {
    std::ofstream os(path, std::ios::binary | std::ios::trunc);
    if (!os) throw IoError("cannot write index file " + path);
    os.write(MAGIC, 8);
    put(os, FILE_VERSION);
    put(os, uint32_t(0));
    put(os, header_len);
    if (header_len) os.write(reinterpret_cast<const char*>(header), (std::streamsize)header_len);
    put(os, idx.n);
    put(os, idx.n_records);
    put(os, idx.n_texts);
    put(os, idx.n_groups);
    put(os, idx.prefix_q);
    os.write(reinterpret_cast<const char*>(idx.C), sizeof(idx.C));
    put_vec(os, idx.text);
    put_vec(os, idx.text_start);
    put_vec(os, idx.text_group);
    put_vec(os, idx.group_of_rec);
    put_vec(os, idx.occ);
    put_vec(os, idx.occ2);
    put_vec(os, idx.occ3);
    put_vec(os, idx.runs);
    put_vec(os, idx.run_label);
    put_vec(os, idx.lab);
    put_vec(os, idx.prefix);
    put_vec(os, idx.prefix1);
    put_vec(os, idx.prefix2);
    if (!os) throw IoError("failed writing index file " + path);
}

void fm_read_header(const std::string& path, std::vector<uint8_t>& header) {
    std::ifstream is(path, std::ios::binary);
    if (!is) throw IoError("cannot open index file " + path);
    read_preamble(is, path, &header);
}

// The arrays are read by several threads at once (positional reads of 8 MiB pieces; the .idx of config 3 is 377 MB,
// whose sequential read was a fifth of a `speq scan` run): a first pass takes each array's count and file offset, the
// arrays are sized in parallel (their zero fill is most of a page-cache read's cost), then the pieces are read.
void fm_load(FmIndex& idx, const std::string& path, std::vector<uint8_t>* header) {
    std::ifstream is(path, std::ios::binary);
    if (!is) throw IoError("cannot open index file " + path);
    read_preamble(is, path, header);
    idx = FmIndex();
    get(is, idx.n);
    get(is, idx.n_records);
    get(is, idx.n_texts);
    get(is, idx.n_groups);
    get(is, idx.prefix_q);
    is.read(reinterpret_cast<char*>(idx.C), sizeof(idx.C));
    const uint64_t lim = uint64_t(1) << 36;
    struct Part {
        uint64_t count = 0, elem = 0, offset = 0;
        std::function<char*(uint64_t)> size;  // resizes the array, returns its bytes
        char* data = nullptr;
    };
    std::vector<Part> parts;
    auto toc = [&](auto& v) {  // the array's count and offset; skip its bytes
        using T = typename std::decay_t<decltype(v)>::value_type;
        Part pt;
        get(is, pt.count);
        if (pt.count > lim) throw IoError("corrupt index file (array too large)");
        pt.elem = sizeof(T);
        pt.offset = (uint64_t)is.tellg();
        pt.size = [&v](uint64_t c) {
            v.resize(c);
            return reinterpret_cast<char*>(v.data());
        };
        is.seekg((std::streamoff)(pt.offset + pt.count * pt.elem));
        if (!is) throw IoError("truncated index file");
        parts.push_back(std::move(pt));
    };
    toc(idx.text);
    toc(idx.text_start);
    toc(idx.text_group);
    toc(idx.group_of_rec);
    toc(idx.occ);
    toc(idx.occ2);
    toc(idx.occ3);
    toc(idx.runs);
    toc(idx.run_label);
    toc(idx.lab);
    toc(idx.prefix);
    toc(idx.prefix1);
    toc(idx.prefix2);
    is.seekg(0, std::ios::end);
    const uint64_t file_len = (uint64_t)is.tellg();
    for (const Part& pt : parts)
        if (pt.offset + pt.count * pt.elem > file_len) throw IoError("truncated index file");
    is.close();
    {
        std::vector<std::thread> ts;
        for (Part& pt : parts) ts.emplace_back([&pt] { pt.data = pt.size(pt.count); });
        for (auto& t : ts) t.join();
    }
    struct Piece {
        char* dst;
        uint64_t off, len;
    };
    std::vector<Piece> pieces;
    const uint64_t PIECE = 8ull << 20;
    for (const Part& pt : parts)
        for (uint64_t b = 0; b < pt.count * pt.elem; b += PIECE)
            pieces.push_back({pt.data + b, pt.offset + b, std::min(PIECE, pt.count * pt.elem - b)});
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw IoError("cannot open index file " + path);
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    const unsigned nt = std::max(1u, std::min<unsigned>(16u, std::thread::hardware_concurrency()));
    {
        std::vector<std::thread> ts;
        for (unsigned t = 0; t < std::min<size_t>(nt, pieces.size()); ++t)
            ts.emplace_back([&] {
                for (size_t i; (i = next.fetch_add(1)) < pieces.size() && !failed.load();) {
                    const Piece& pc = pieces[i];
                    for (uint64_t done = 0; done < pc.len;) {
                        const ssize_t r = ::pread(fd, pc.dst + done, pc.len - done, (off_t)(pc.off + done));
                        if (r <= 0) {
                            if (r < 0 && errno == EINTR) continue;
                            failed = true;
                            break;
                        }
                        done += (uint64_t)r;
                    }
                }
            });
        for (auto& t : ts) t.join();
    }
    ::close(fd);
    if (failed) throw IoError("cannot read index file " + path);
    const uint64_t nb = idx.n_blocks();
    if (idx.text.size() != idx.n || idx.text_start.size() != (uint64_t)idx.n_texts + 1 ||
        idx.text_group.size() != idx.n_texts || idx.occ.size() != nb * 5 || (!idx.occ2.empty() && idx.occ2.size() != nb * 16) ||
        (!idx.occ3.empty() && (idx.occ3.size() != nb * 64 || idx.occ2.empty())) || (!idx.lab.empty() && idx.lab.size() != idx.n) ||
        idx.runs.size() != nb || idx.prefix_q > MAX_PREFIX_Q ||
        idx.prefix.size() != (idx.prefix_q ? 2 * (uint64_t(1) << (2 * idx.prefix_q)) : 0) ||
        idx.prefix1.size() != (idx.prefix_q >= 2 ? 2 * (uint64_t(1) << (2 * (idx.prefix_q - 1))) : 0) ||
        idx.prefix2.size() != (idx.prefix_q >= 3 ? 2 * (uint64_t(1) << (2 * (idx.prefix_q - 2))) : 0) ||
        idx.n_groups == 0)
        throw IoError("inconsistent index file " + path);
}

}  // namespace speq
