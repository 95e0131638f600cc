// FASTQ (plain or gzip) -> pinned slots -> GPU scan: the streaming front end of speq_scan_fastq.
//
// Replaces seqan3::sequence_file_input + views::async_input_buffer (/root/reference/src/fm_scanner.cpp:138-141;
// paired: views::zip(fin1, fin2), :651-655, which stops at the shorter file). One reader thread decompresses (zlib
// gzread, transparent for plain files) and cuts record-aligned text blocks; parser threads turn blocks into
// {bases, qualities, offsets} directly inside pinned pipeline slots and submit them (pipeline.cpp), so parsing,
// PCIe copies and the kernel overlap.
//
// FASTQ grammar (same as FastqReader in host_io.cpp): blank lines between records are skipped; a record is
// '@' header, sequence lines up to a line starting with '+', then quality lines until as many quality characters
// as bases have been read; whitespace and digits inside sequence lines are dropped, whitespace inside quality
// lines is dropped; a FASTA file is rejected (qualities are required).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>
#include <emmintrin.h>

#include <cerrno>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "capi_internal.hpp"
#include "scan_internal.hpp"

namespace {

using speq::IoError;

// Decompressed byte source: plain files through read(2), gzip (magic 1f 8b) through zlib.
// BGZF (blocked gzip, as written by bgzip): a series of independent gzip members whose headers carry the member size
// ("BC" extra subfield) and whose footers carry the uncompressed size, so members can be inflated in parallel
// straight into their final positions. Plain gzip streams have no such index and are inflated sequentially.
class Bgzf {
public:
    Bgzf(const std::string& path, int fd, uint32_t threads) : path_(path), threads_(std::max<uint32_t>(1, threads)) {
        struct stat st {};
        if (::fstat(fd, &st) != 0) throw IoError("cannot stat " + path);
        size_ = (size_t)st.st_size;
        map_ = static_cast<const uint8_t*>(::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0));
        if (map_ == MAP_FAILED) {
            map_ = nullptr;
            throw IoError("cannot map " + path);
        }
        (void)::madvise((void*)map_, size_, MADV_SEQUENTIAL);
    }
    ~Bgzf() {
        if (map_) ::munmap((void*)map_, size_);
    }
    // True when the file starts with a BGZF member header.
    static bool is_bgzf(const uint8_t* h, size_t n) {
        if (n < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return false;
        const size_t xlen = h[10] | (h[11] << 8);
        for (size_t i = 12; i + 4 <= 12 + xlen && i + 4 <= n;) {
            const size_t slen = h[i + 2] | (h[i + 3] << 8);
            if (h[i] == 'B' && h[i + 1] == 'C' && slen == 2) return true;
            i += 4 + slen;
        }
        return false;
    }
    // Inflates the next members whose uncompressed sizes fit in n bytes (at least one) into dst, in parallel.
    size_t read(char* dst, size_t n) {
        struct Member {
            size_t cpos, csize, dpos, dsize;
        };
        std::vector<Member> batch;
        size_t out = 0;
        while (pos_ < size_) {
            const Next m = next_member(pos_);
            if (out + m.dsize > n) {
                // the caller's buffer is full; members hold at most 64 KiB, so a larger buffer always takes one
                if (batch.empty() && n >= 65536) throw IoError("BGZF member larger than 64 KiB in " + path_);
                break;
            }
            batch.push_back({m.cpos, m.csize, out, m.dsize});
            out += m.dsize;
            pos_ += m.csize;
        }
        if (batch.empty()) return 0;
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        auto work = [&] {
            z_stream z;
            std::memset(&z, 0, sizeof(z));
            if (inflateInit2(&z, -15) != Z_OK) {
                bad = true;
                return;
            }
            for (size_t i; (i = next++) < batch.size() && !bad;) {
                const Member& m = batch[i];
                const uint8_t* h = map_ + m.cpos;
                const size_t xlen = h[10] | (h[11] << 8);
                const size_t hdr = 12 + xlen;
                if (m.csize < hdr + 8) {
                    bad = true;
                    break;
                }
                (void)inflateReset(&z);
                z.next_in = const_cast<Bytef*>(h + hdr);
                z.avail_in = (uInt)(m.csize - hdr - 8);
                z.next_out = reinterpret_cast<Bytef*>(dst + m.dpos);
                z.avail_out = (uInt)m.dsize;
                const int rc = inflate(&z, Z_FINISH);
                const uint8_t* f = h + m.csize - 8;
                const uint32_t crc = f[0] | (f[1] << 8) | (f[2] << 16) | ((uint32_t)f[3] << 24);
                if (rc != Z_STREAM_END || z.total_out != m.dsize ||
                    crc32(0L, reinterpret_cast<const Bytef*>(dst + m.dpos), (uInt)m.dsize) != crc)
                    bad = true;
            }
            inflateEnd(&z);
        };
        const uint32_t t = (uint32_t)std::min<size_t>(threads_, batch.size());
        std::vector<std::thread> pool;
        for (uint32_t i = 1; i < t; ++i) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();
        if (bad) throw IoError("corrupt BGZF member in " + path_);
        return out;
    }

private:
    struct Next {
        size_t cpos, csize, dsize;
    };
    Next next_member(size_t p) const {
        const uint8_t* h = map_ + p;
        if (size_ - p < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4))
            throw IoError("not a BGZF member at byte " + std::to_string(p) + " of " + path_);
        const size_t xlen = h[10] | (h[11] << 8);
        size_t bsize = 0;
        for (size_t i = 12; i + 4 <= 12 + xlen;) {
            const size_t slen = h[i + 2] | (h[i + 3] << 8);
            if (h[i] == 'B' && h[i + 1] == 'C' && slen == 2) bsize = (size_t)(h[i + 4] | (h[i + 5] << 8)) + 1;
            i += 4 + slen;
        }
        if (bsize < 12 + xlen + 8 || p + bsize > size_) throw IoError("corrupt BGZF header in " + path_);
        const uint8_t* f = h + bsize - 4;
        const size_t isize = f[0] | (f[1] << 8) | (f[2] << 16) | ((size_t)f[3] << 24);
        return {p, bsize, isize};
    }
    std::string path_;
    uint32_t threads_;
    const uint8_t* map_ = nullptr;
    size_t size_ = 0, pos_ = 0;
};

// Decompressed byte source: plain files through read(2), BGZF through parallel member inflation, other gzip
// (magic 1f 8b) through zlib.
class Source {
public:
    explicit Source(const std::string& path, uint32_t threads = 1) : path_(path) {
        fd_ = ::open(path.c_str(), O_RDONLY);
        if (fd_ < 0) throw IoError("cannot open reads file " + path);
        unsigned char head[64] = {0};
        const ssize_t m = ::pread(fd_, head, sizeof(head), 0);
        if (m >= 2 && head[0] == 0x1f && head[1] == 0x8b) {
            if (Bgzf::is_bgzf(head, (size_t)m)) {
                bgzf_ = std::make_unique<Bgzf>(path, fd_, threads);
                return;
            }
            gz_ = gzdopen(fd_, "rb");
            if (!gz_) throw IoError("cannot open gzip stream " + path);
            fd_ = -1;  // owned by gz_
            gzbuffer(gz_, 1u << 20);
        } else {
            (void)::posix_fadvise(fd_, 0, 0, POSIX_FADV_SEQUENTIAL);
        }
    }
    ~Source() {
        bgzf_.reset();
        if (gz_) gzclose(gz_);
        if (fd_ >= 0) ::close(fd_);
    }
    size_t read(char* dst, size_t n) {
        if (bgzf_) {
            size_t got = 0;
            while (got < n) {
                const size_t r = bgzf_->read(dst + got, n - got);
                if (r == 0) break;
                got += r;
            }
            return got;
        }
        size_t got = 0;
        while (got < n) {
            const size_t want = std::min<size_t>(n - got, 1u << 30);
            if (gz_) {
                const int r = gzread(gz_, dst + got, (unsigned)want);
                if (r < 0) {
                    int err = 0;
                    const char* msg = gzerror(gz_, &err);
                    throw IoError("error reading " + path_ + ": " + (msg ? msg : "zlib error"));
                }
                if (r == 0) break;
                got += (size_t)r;
            } else {
                const ssize_t r = ::read(fd_, dst + got, want);
                if (r < 0) {
                    if (errno == EINTR) continue;
                    throw IoError("error reading " + path_ + ": " + std::strerror(errno));
                }
                if (r == 0) break;
                got += (size_t)r;
            }
        }
        return got;
    }
    const std::string& path() const { return path_; }
    bool plain() const { return gz_ == nullptr && !bgzf_; }
    int fd() const { return fd_; }

private:
    int fd_ = -1;
    gzFile gz_ = nullptr;
    std::unique_ptr<Bgzf> bgzf_;
    std::string path_;
};

inline bool is_space(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
inline bool is_seq_char(unsigned char c) { return !is_space(c) && !(c >= '0' && c <= '9'); }

// Line [b, e) of data starting at pos, '\n' excluded; trailing '\r's excluded from e. Returns false if no complete
// line is available (a final unterminated line counts as complete only at end of input).
inline bool get_line(const char* data, size_t len, size_t& pos, bool eof, size_t& b, size_t& e) {
    if (pos >= len) return false;
    const char* nl = static_cast<const char*>(std::memchr(data + pos, '\n', len - pos));
    size_t stop, next;
    if (nl) {
        stop = (size_t)(nl - data);
        next = stop + 1;
    } else {
        if (!eof) return false;
        stop = len;
        next = len;
    }
    b = pos;
    e = stop;
    while (e > b && data[e - 1] == '\r') --e;
    pos = next;
    return true;
}

size_t count_seq(const char* p, size_t n) {
    size_t c = 0;
    for (size_t i = 0; i < n; ++i) c += is_seq_char((unsigned char)p[i]);
    return c;
}
size_t count_nonspace(const char* p, size_t n) {
    size_t c = 0;
    for (size_t i = 0; i < n; ++i) c += !is_space((unsigned char)p[i]);
    return c;
}

enum ScanResult { REC_COMPLETE, REC_NEED_MORE, REC_NONE };

// Finds the end of the record starting at pos (blank lines first), validating the general grammar.
ScanResult scan_record(const char* data, size_t len, size_t pos, bool eof, size_t& end, const std::string& path) {
    size_t b = 0, e = 0;
    for (;;) {
        if (!get_line(data, len, pos, eof, b, e)) return eof ? REC_NONE : REC_NEED_MORE;
        if (e > b) break;
    }
    if (data[b] != '@') {
        if (data[b] == '>') throw IoError("reads must be FASTQ (qualities are required): " + path);
        throw IoError("malformed FASTQ record header in " + path + ": " + std::string(data + b, std::min<size_t>(e - b, 80)));
    }
    size_t seq = 0, qual = 0;
    for (;;) {
        if (!get_line(data, len, pos, eof, b, e)) {
            if (eof) throw IoError("truncated FASTQ record (no '+' line) in " + path);
            return REC_NEED_MORE;
        }
        if (e > b && data[b] == '+') break;
        seq += count_seq(data + b, e - b);
    }
    while (qual < seq) {
        if (!get_line(data, len, pos, eof, b, e)) {
            if (eof) break;
            return REC_NEED_MORE;
        }
        qual += count_nonspace(data + b, e - b);
    }
    if (qual != seq) throw IoError("FASTQ record with sequence/quality length mismatch in " + path);
    end = pos;
    return REC_COMPLETE;
}

// Four-line record (@header / bases / '+' / qualities of the same raw length) found with four memchr and no
// per-byte work; anything else (blank lines, wrapped records, CR-only oddities) goes through scan_record. The
// parser re-checks every record against the general grammar (parse_record), so a fast cut never changes results.
inline bool fast_record(const char* data, size_t len, size_t pos, bool eof, size_t& end, size_t& seq_len) {
    if (pos >= len || data[pos] != '@') return false;
    size_t nl[4];
    size_t p = pos;
    for (int i = 0; i < 4; ++i) {
        const char* q = p < len ? static_cast<const char*>(std::memchr(data + p, '\n', len - p)) : nullptr;
        if (!q) {
            if (i < 3 || !eof || p >= len) return false;
            nl[i] = len;  // last line unterminated at end of input
            p = len;
            break;
        }
        nl[i] = (size_t)(q - data);
        p = nl[i] + 1;
        if (i == 0 && p < len && data[p] == '+') return false;  // a base line opening with '+' is the separator
        if (i == 1 && (p >= len || data[p] != '+')) return false;
    }
    auto trimmed = [&](size_t b, size_t e) {
        while (e > b && data[e - 1] == '\r') --e;
        return e - b;
    };
    const size_t l2 = trimmed(nl[0] + 1, nl[1]), l4 = trimmed(nl[2] + 1, nl[3]);
    if (l2 != l4 || trimmed(pos, nl[0]) == 0) return false;
    end = p;
    seq_len = l2;
    return true;
}

// A decompressed buffer, or the whole mapping of a plain file; blocks keep it alive until parsed. Bytes [0, len)
// are immutable once written.
struct Buf {
    std::unique_ptr<char[]> own;
    char* ptr = nullptr;
    size_t cap = 0, len = 0;
    void* map = nullptr;
    size_t map_len = 0;
    bool registered = false;  // page-locked for direct DMA (SPEQ_FASTQ_DIRECT=2); every copy from it has completed
    ~Buf() {                  // before the last block releases it (run_stream drains the copies first)
        if (registered) speq::host_unregister(map);
        if (map) ::munmap(map, map_len);
    }
    char* data() const { return ptr; }
};

struct Block {
    std::shared_ptr<Buf> buf;
    size_t begin = 0, end = 0;
    uint64_t n = 0;
    bool simple = true;   // every record took the four-line fast path (eligible for GPU parsing)
    uint64_t bases = 0;   // raw base-line bytes of those records
    const char* data() const { return buf ? buf->data() + begin : nullptr; }
    size_t size() const { return end - begin; }
};

// Cuts record-aligned blocks out of one decompressed stream without copying them.
class Cutter {
public:
    // Plain files are mapped whole (no read copies; parsers read the page cache directly); gzip is inflated into
    // 64 MiB buffers.
    // `populate` maps every page up front (one thread); without it the parsers fault their own blocks in parallel,
    // which pays off when the blocks are cut without reading the file first (run_stream's split mode).
    explicit Cutter(const std::string& path, uint32_t threads = 1, bool populate = true) : src_(path, threads) {
        if (!src_.plain()) return;
        struct stat st {};
        if (::fstat(src_.fd(), &st) != 0 || !S_ISREG(st.st_mode)) return;  // pipes etc.: read path
        auto b = std::make_shared<Buf>();
        if (st.st_size > 0) {
            const int flags = MAP_PRIVATE | (populate ? MAP_POPULATE : 0);
            void* m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, flags, src_.fd(), 0);
            if (m == MAP_FAILED) return;
            (void)::madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
            b->map = m;
            b->map_len = (size_t)st.st_size;
            b->ptr = static_cast<char*>(m);
            b->cap = b->len = (size_t)st.st_size;
        }
        cur_ = std::move(b);
        eof_ = true;
    }
    // Up to max_records complete records, stopping after the record that reaches max_bytes.
    Block next(uint64_t max_records, uint64_t max_bytes) {
        uint64_t n = 0, bases = 0;
        bool simple = true;
        if (!cur_) grow(0);
        size_t pos = pos_;
        while (n < max_records && (n == 0 || pos - pos_ < max_bytes)) {
            const char* data = cur_->data();
            size_t end = 0, seq_len = 0;
            if (fast_record(data, cur_->len, pos, eof_, end, seq_len)) {
                pos = end;
                ++n;
                bases += seq_len;
                continue;
            }
            const ScanResult r = scan_record(data, cur_->len, pos, eof_, end, src_.path());
            if (r == REC_COMPLETE) {
                pos = end;
                ++n;
                simple = false;
            } else if (r == REC_NONE) {
                break;
            } else {
                pos = refill(pos);
            }
        }
        Block blk{cur_, pos_, pos, n, simple, bases};
        pos_ = pos;
        return blk;
    }

    // The whole file when it is mapped and nothing has been cut yet, else null.
    std::shared_ptr<Buf> mapping() const { return (eof_ && cur_ && cur_->map && pos_ == 0) ? cur_ : nullptr; }

private:
    static constexpr size_t BUF_BYTES = 64u << 20, READ_BYTES = 16u << 20;
    // Makes room for READ_BYTES more input; moves the unconsumed tail [pos_, len) into a fresh buffer when the
    // current one is full (blocks still reference the old one). Returns `pos` translated into the new buffer.
    size_t refill(size_t pos) {
        if (cur_->cap - cur_->len < READ_BYTES) pos = grow(pos);
        const size_t r = src_.read(cur_->data() + cur_->len, std::min(READ_BYTES, cur_->cap - cur_->len));
        cur_->len += r;
        if (r == 0) eof_ = true;
        return pos;
    }
    size_t grow(size_t pos) {
        auto nb = std::make_shared<Buf>();
        const size_t tail = cur_ ? cur_->len - pos_ : 0;
        nb->cap = std::max(BUF_BYTES, 2 * tail + READ_BYTES);
        nb->own.reset(new char[nb->cap]);
        nb->ptr = nb->own.get();
        if (tail) std::memcpy(nb->ptr, cur_->data() + pos_, tail);
        nb->len = tail;
        const size_t shift = pos_;
        cur_ = std::move(nb);
        pos_ = 0;
        return pos - shift;
    }
    Source src_;
    std::shared_ptr<Buf> cur_;
    size_t pos_ = 0;
    bool eof_ = false;
};

// Parses the record at pos of a block into (seq, qual) at `out` with the general grammar; returns the new out.
// Throws when the record is not what the cutter saw (only possible for pathological files; see fast_record).
uint64_t parse_record(const char* data, size_t len, size_t& pos, uint8_t* seq, uint8_t* qual, uint64_t out,
                      const char* path) {
    auto line = [&](size_t& b, size_t& e) {
        if (!get_line(data, len, pos, true, b, e))
            throw IoError(std::string("irregular FASTQ record (sequence/quality line layout) in ") + path);
    };
    size_t b = 0, e = 0;
    do {
        line(b, e);
    } while (e == b);
    uint64_t s = out;
    for (;;) {
        line(b, e);
        if (e > b && data[b] == '+') break;
        const size_t n = e - b;
        std::memcpy(seq + s, data + b, n);  // fast path: no blanks/digits inside the line
        if (count_seq(data + b, n) == n) {
            s += n;
        } else {
            for (size_t i = b; i < e; ++i)
                if (is_seq_char((unsigned char)data[i])) seq[s++] = (uint8_t)data[i];
        }
    }
    uint64_t q = out;
    while (q < s) {  // every non-blank character of a quality line counts, as in scan_record
        line(b, e);
        const size_t n = e - b, c = count_nonspace(data + b, n);
        if (q + c > s) throw IoError(std::string("FASTQ record with sequence/quality length mismatch in ") + path);
        if (c == n) {
            std::memcpy(qual + q, data + b, n);
        } else {
            uint64_t w = q;
            for (size_t i = b; i < e; ++i)
                if (!is_space((unsigned char)data[i])) qual[w++] = (uint8_t)data[i];
        }
        q += c;
    }
    return s;
}

// memcpy that also counts the '\n' bytes it copies (one pass over the page cache instead of two).
uint64_t copy_count_nl(char* dst, const char* src, size_t n) {
    const __m128i nl = _mm_set1_epi8('\n');
    uint64_t c = 0;
    size_t i = 0;
    // non-temporal stores into the (16-B aligned) pinned slot when SPEQ_NT_COPY is not 0: the slot is only read by
    // the DMA engine, and streaming stores skip the read-for-ownership of every destination line (host memory
    // bandwidth is what bounds this path)
    static const bool nt = [] {
        const char* e = std::getenv("SPEQ_NT_COPY");
        return !(e && e[0] == '0');
    }();
    const bool stream = nt && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        if (stream) {
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), d);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), e);
        } else {
            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i), a);
            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 32), d);
            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 48), e);
        }
        const uint64_t m = (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(a, nl)) |
                           (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(b, nl)) << 16 |
                           (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(d, nl)) << 32 |
                           (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(e, nl)) << 48;
        c += (uint64_t)__builtin_popcountll(m);
    }
    for (; i < n; ++i) c += (dst[i] = src[i]) == '\n';
    if (stream) _mm_sfence();  // the streamed lines are globally visible before the slot is submitted
    return c;
}

// A mapped single-end file whose records are not all four-line ones: the parallel cut below cannot be trusted, and
// the stream restarts with the sequential cutter.
struct NotSimple : std::runtime_error {
    NotSimple() : std::runtime_error("FASTQ layout needs the sequential cutter") {}
};

// First header line at or after byte t (t > 0): a line starting with '@' whose next-but-one line starts with '+'.
// In a file of four-line records only headers qualify (a quality line starting with '@' is followed by a header
// and then a sequence line); returns len when no header starts before the end, or throws NotSimple after 1 MiB.
size_t find_cut(const char* data, size_t len, size_t t) {
    const char* q = static_cast<const char*>(std::memchr(data + t - 1, '\n', len - (t - 1)));
    size_t c = q ? (size_t)(q - data) + 1 : len;
    while (c < len) {
        if (c - t > (1u << 20)) throw NotSimple();
        const char* n1 = static_cast<const char*>(std::memchr(data + c, '\n', len - c));
        if (!n1) return len;
        if (data[c] == '@') {
            const size_t l2 = (size_t)(n1 - data) + 1;
            const char* n2 = l2 < len ? static_cast<const char*>(std::memchr(data + l2, '\n', len - l2)) : nullptr;
            if (!n2) return len;
            if ((size_t)(n2 - data) + 1 < len && n2[1] == '+') return c;
        }
        c = (size_t)(n1 - data) + 1;
    }
    return len;
}

struct Work {
    Block b1, b2;
    uint64_t n = 0;      // records (pairs when paired) to parse
    bool split = false;  // cut by find_cut: records not yet counted or checked
    uint64_t seq = 0;    // block number in file order (the rank sharding deals blocks by it)
};

// Which blocks this process scans: block b belongs to shard b % n (one process per GPU, `speq scan` under a
// launcher that sets RANK / WORLD_SIZE). The blocks are cut the same way on every rank, so the shards partition the
// records. n = 1: every block.
struct ShardSel {
    uint32_t index = 0, n = 1;
    bool mine(uint64_t block) const { return n <= 1 || block % n == index; }
};

struct Shared {
    std::mutex mu;
    std::condition_variable cv_put, cv_get;
    std::deque<Work> q;
    size_t max_q = 4;
    bool done = false;
    std::atomic<bool> failed{false};
    std::string error;
    bool io_error = false, retry = false;
    std::atomic<uint64_t> records{0}, bases{0}, batches{0};
    void fail(const std::string& msg, bool io, bool not_simple = false) {
        std::lock_guard<std::mutex> lk(mu);
        if (!failed.exchange(true)) {
            error = msg;
            io_error = io;
            retry = not_simple;
        }
        done = true;
        cv_put.notify_all();
        cv_get.notify_all();
    }
};

void check_rc(int rc) {
    if (rc != SPEQ_OK) throw speq::DeviceError(speq_last_error());
}


// Where parsed blocks go: pinned pipeline slots (speq_scan_fastq) or host memory (speq_fastq_checksum, CPU tests).
struct Sink {
    virtual ~Sink() = default;
    virtual void acquire(speq_slot& s, uint64_t bytes, uint64_t records) = 0;
    // a slot for raw text only (s.seq; submit_raw or submit(s, 0) next)
    virtual void acquire_raw(speq_slot& s, uint64_t bytes) { acquire(s, bytes, 1); }
    virtual void submit(const speq_slot& s, uint64_t records) = 0;  // records == 0 releases the slot
    // raw four-line FASTQ text (file 1's block, then file 2's) in s.seq, n records per file
    // host1 / host2 non-null: the blocks are copied from there (the file's mapping), not from s.seq
    virtual void submit_raw(const speq_slot& s, uint64_t len1, uint64_t len2, uint64_t n, bool paired,
                            const char* host1 = nullptr, const char* host2 = nullptr) {
        (void)s; (void)len1; (void)len2; (void)n; (void)paired; (void)host1; (void)host2;
        throw std::logic_error("this sink does not parse raw FASTQ");
    }
    // waits until every H2D copy issued so far has completed (before a registered mapping is released)
    virtual void drain_copies() {}
    // records packed by pack_records (s.offsets filled; 3 bits per base when `three`, else one byte)
    virtual void submit_packed(const speq_slot& s, uint64_t records, bool three) {
        (void)s; (void)records; (void)three;
        throw std::logic_error("this sink does not take packed records");
    }
};

// Host packing of four-line FASTQ blocks (SPEQ_FASTQ_PACK=1; by default raw text goes to the GPU parser): 3 bits per
// base in global mode, one byte per base in local mode (pipeline.cpp's formats), so the PCIe bytes per 150-bp record
// drop from ~340 (raw text) to 56 or 150, at ~180 ns of host time per record.
struct PackMode {
    int kind = 0;         // 0 off, 1 one byte per base, 2 three bits per base
    uint32_t cutoff = 30;
};

// every byte of [p, p + n) >= lo (unsigned)
inline bool all_at_least(const char* p, size_t n, uint8_t lo) {
    const __m128i l = _mm_set1_epi8((char)lo);
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i));
        if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_max_epu8(x, l), x)) != 0xFFFF) return false;
    }
    for (; i < n; ++i)
        if ((uint8_t)p[i] < lo) return false;
    return true;
}

// Newline offsets of [b, e) of d (absolute), appended to out; one SSE2 pass (movemask + bit scan).
void newlines(const char* d, size_t b, size_t e, std::vector<uint32_t>& out) {
    const __m128i nl = _mm_set1_epi8('\n');
    size_t i = b;
    for (; i + 16 <= e; i += 16) {
        uint32_t m = (uint32_t)_mm_movemask_epi8(
            _mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(d + i)), nl));
        while (m) {
            out.push_back((uint32_t)(i + (uint32_t)__builtin_ctz(m) - b));
            m &= m - 1;
        }
    }
    for (; i < e; ++i)
        if (d[i] == '\n') out.push_back((uint32_t)(i - b));
}

// Packs n four-line records from [b1, e1) of d1 (and, paired, n from [b2, e2) of d2, interleaved as mates) into
// slot s (offsets + packed bases). False when a record is not a clean four-line record or the records do not end
// the range exactly (a header not opening with '@', a separator not opening with '+', base and quality lines of
// different lengths, a base line holding anything below 'A' — blanks and digits the grammar drops —, a quality
// line holding blanks): the caller then takes the general path, which parses such records by the grammar. The
// lines come from one newline pass per block; wide loads may read up to 31 bytes past a line, never past the end
// of the buffer (`lim`).
bool pack_records(const char* d1, size_t b1, size_t e1, size_t lim1, const char* d2, size_t b2, size_t e2,
                  size_t lim2, uint64_t n, bool paired, const PackMode& pm, speq_slot& s, uint64_t raw_bytes,
                  uint64_t& bases) {
    const bool three = pm.kind == 2;
    const uint64_t nw_max = raw_bytes / 32 + 2;  // base words the block can need
    uint64_t* codes = reinterpret_cast<uint64_t*>(s.seq);
    uint32_t* bad_max = reinterpret_cast<uint32_t*>(s.seq + nw_max * 8);
    if (three) std::memset(s.seq, 0, nw_max * 12);
    thread_local std::vector<uint32_t> nl1, nl2;
    nl1.clear();
    nl2.clear();
    if (e1 - b1 >= (1ull << 32) || (paired && e2 - b2 >= (1ull << 32))) return false;
    newlines(d1, b1, e1, nl1);
    if (paired) newlines(d2, b2, e2, nl2);
    // an unterminated last line at the end of the input counts as terminated there
    if (e1 > b1 && d1[e1 - 1] != '\n') {
        if (e1 != lim1) return false;
        nl1.push_back((uint32_t)(e1 - b1));
    }
    if (paired && e2 > b2 && d2[e2 - 1] != '\n') {
        if (e2 != lim2) return false;
        nl2.push_back((uint32_t)(e2 - b2));
    }
    if (nl1.size() != 4 * n || (paired && nl2.size() != 4 * n)) return false;
    uint64_t at = 0, r = 0;
    s.offsets[0] = 0;
    auto one = [&](const char* d, size_t b, size_t lim, const std::vector<uint32_t>& nl, uint64_t i) -> bool {
        const size_t h = i ? b + nl[4 * i - 1] + 1 : b;  // header line start
        const size_t l0 = b + nl[4 * i], l1 = b + nl[4 * i + 1], l2 = b + nl[4 * i + 2], l3 = b + nl[4 * i + 3];
        if (d[h] != '@' || d[l1 + 1] != '+' || d[l0 + 1] == '+') return false;
        size_t hl = l0;
        while (hl > h && d[hl - 1] == '\r') --hl;
        if (hl <= h + 0) return false;  // empty header line (only '@' is fine: it is one byte)
        size_t se = l1, qe = l3;
        while (se > l0 + 1 && d[se - 1] == '\r') --se;
        while (qe > l2 + 1 && d[qe - 1] == '\r') --qe;
        const size_t L = se - (l0 + 1);
        if (qe - (l2 + 1) != L) return false;
        const char* sq = d + l0 + 1;
        const char* qq = d + l2 + 1;
        if (!all_at_least(sq, L, 'A') || !all_at_least(qq, L, 0x21)) return false;
        const bool wide = l2 + 1 + L + 32 <= lim;  // a 32-byte load at the quality tail stays in the buffer
        if (three)
            speq::pack_bases3_append(codes, bad_max, at, reinterpret_cast<const uint8_t*>(sq),
                                     reinterpret_cast<const uint8_t*>(qq), L, pm.cutoff, wide);
        else
            speq::pack_bases(s.seq + at, reinterpret_cast<const uint8_t*>(sq), reinterpret_cast<const uint8_t*>(qq), L);
        at += L;
        s.offsets[++r] = at;
        return true;
    };
    for (uint64_t i = 0; i < n; ++i) {
        if (!one(d1, b1, lim1, nl1, i)) return false;
        if (paired && !one(d2, b2, lim2, nl2, i)) return false;
    }
    if (three) {  // the bad words follow the code words of the bases actually packed
        const uint64_t nw = (at + 31) / 32;
        std::memmove(s.seq + nw * 8, bad_max, nw * 4);
    }
    bases = at;
    return true;
}

// Slots of one or more pipelines (one per GPU replica), dealt in turn: with equal GPUs every replica scans every
// n-th block. The pipeline index travels in the slot id (slot * n + pipeline).
struct PipelineSink final : Sink {
    std::vector<speq_pipeline*> pls;
    std::atomic<uint64_t> next{0};
    explicit PipelineSink(std::vector<speq_pipeline*> p) : pls(std::move(p)) {}
    uint32_t pick() { return (uint32_t)(next++ % pls.size()); }
    speq_pipeline* of(int32_t slot) const { return pls[(uint32_t)slot % pls.size()]; }
    int32_t local(int32_t slot) const { return slot / (int32_t)pls.size(); }
    int32_t global(int32_t slot, uint32_t i) const { return slot * (int32_t)pls.size() + (int32_t)i; }
    void acquire(speq_slot& s, uint64_t bytes, uint64_t records) override {
        const uint32_t i = pick();
        speq_pipeline* pl = pls[i];
        check_rc(speq_pipeline_acquire(pl, &s));
        if (bytes > s.cap_bytes || records > s.cap_records) {
            const int rc = speq_pipeline_reserve(pl, &s, bytes, records);
            if (rc != SPEQ_OK) {
                (void)speq_pipeline_submit(pl, s.slot, 0);
                check_rc(rc);
            }
        }
        s.slot = global(s.slot, i);
    }
    void acquire_raw(speq_slot& s, uint64_t bytes) override {
        const uint32_t i = pick();
        s = speq_slot{};
        s.slot = global(speq::pipeline_acquire_raw(pls[i], bytes, &s.seq), i);
        s.cap_bytes = bytes;
    }
    void submit(const speq_slot& s, uint64_t records) override {
        check_rc(speq_pipeline_submit(of(s.slot), local(s.slot), records));
    }
    void submit_raw(const speq_slot& s, uint64_t len1, uint64_t len2, uint64_t n, bool paired, const char* host1,
                    const char* host2) override {
        static std::atomic<bool> first{true};
        if (first.exchange(false)) speq::startup_trace("stream: first block submitted");
        speq::pipeline_submit_raw(of(s.slot), local(s.slot), len1, len2, n, paired,
                                  reinterpret_cast<const uint8_t*>(host1), reinterpret_cast<const uint8_t*>(host2));
    }
    void drain_copies() override {
        for (speq_pipeline* pl : pls) speq::pipeline_sync_copies(pl);
    }
    void submit_packed(const speq_slot& s, uint64_t records, bool three) override {
        if (three) speq::pipeline_submit_packed3(of(s.slot), local(s.slot), records);
        else speq::pipeline_submit_packed(of(s.slot), local(s.slot), records);
    }
};

// Order-independent digest of the parsed records (sum over records of a 64-bit hash of length, bases and
// qualities), so CPU tests can check the reader/parser without a GPU.
struct ChecksumSink final : Sink {
    std::mutex mu;
    std::atomic<uint64_t> digest{0};
    struct Held {
        std::vector<uint8_t> seq, qual;
        std::vector<uint64_t> off;
    };
    std::vector<std::unique_ptr<Held>> held;
    std::vector<int> free_ids;
    void acquire(speq_slot& s, uint64_t bytes, uint64_t records) override {
        std::lock_guard<std::mutex> lk(mu);
        int id;
        if (free_ids.empty()) {
            id = (int)held.size();
            held.push_back(std::make_unique<Held>());
        } else {
            id = free_ids.back();
            free_ids.pop_back();
        }
        Held& h = *held[(size_t)id];
        h.seq.resize(std::max<uint64_t>(bytes, 1));
        h.qual.resize(std::max<uint64_t>(bytes, 1));
        h.off.resize(records + 1);
        s.seq = h.seq.data();
        s.qual = h.qual.data();
        s.offsets = h.off.data();
        s.cap_bytes = bytes;
        s.cap_records = records;
        s.slot = id;
    }
    static uint64_t mix(uint64_t z) {
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    }
    void submit(const speq_slot& s, uint64_t records) override {
        uint64_t acc = 0;
        for (uint64_t r = 0; r < records; ++r) {
            uint64_t h = 0x9e3779b97f4a7c15ULL ^ (s.offsets[r + 1] - s.offsets[r]);
            for (uint64_t i = s.offsets[r]; i < s.offsets[r + 1]; ++i)
                h = (h ^ ((uint64_t)s.seq[i] << 8 | s.qual[i])) * 0x100000001b3ULL;
            acc += mix(h);
        }
        digest += acc;
        std::lock_guard<std::mutex> lk(mu);
        free_ids.push_back(s.slot);
    }
};

// Pinned slot size of speq_scan_fastq's pipeline: a block pair of up to 12 MiB per file plus one record usually
// fits (larger blocks grow their slot once: speq_pipeline_reserve).
constexpr uint64_t SLOT_BYTES = 16ull << 20;
// One replica's slot count of a FASTQ stream with `threads` parsers (scan_fastq_impl, n_dev == 1)
uint32_t stream_slots(uint32_t threads) {
    const uint32_t n_parsers = std::max<uint32_t>(1, std::min<uint32_t>(threads ? threads : 1, 64));
    const char* sm = std::getenv("SPEQ_STREAM_SLOTS_MAX");
    const uint32_t slots_max = sm && *sm ? (uint32_t)std::max(3l, std::min(64l, std::atol(sm))) : 18u;
    return std::min<uint32_t>(n_parsers + 2, slots_max);
}

struct StreamTotals {
    uint64_t records = 0, bases = 0, batches = 0;
};

// Offset just past the k-th '\n' of [p, p + n) (k >= 1), or n when there are fewer.
size_t skip_lines(const char* p, size_t n, uint64_t k) {
    const __m128i nl = _mm_set1_epi8('\n');
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const uint32_t m = (uint32_t)_mm_movemask_epi8(
            _mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)), nl));
        const uint32_t c = (uint32_t)__builtin_popcount(m);
        if (c < k) {
            k -= c;
            continue;
        }
        uint32_t mm = m;
        for (uint64_t j = 1; j < k; ++j) mm &= mm - 1;
        return i + (size_t)__builtin_ctz(mm) + 1;
    }
    for (; i < n; ++i)
        if (p[i] == '\n' && --k == 0) return i + 1;
    return n;
}

uint64_t count_nl(const char* p, size_t n) {
    const __m128i nl = _mm_set1_epi8('\n');
    uint64_t c = 0;
    size_t i = 0;
    for (; i + 16 <= n; i += 16)
        c += (uint64_t)__builtin_popcount((uint32_t)_mm_movemask_epi8(
            _mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)), nl)));
    for (; i < n; ++i) c += p[i] == '\n';
    return c;
}

// Block bounds of a mapped file for the parallel cut: 0, guessed record starts ~32 k records apart, len.
std::vector<size_t> split_bounds(const char* data, size_t len, uint64_t block_records, uint64_t block_bytes) {
    uint64_t target = block_bytes;
    size_t p = 0, end = 0, sl = 0;
    uint32_t i = 0;
    for (; i < 256 && fast_record(data, len, p, true, end, sl); ++i) p = end;
    if (i == 0) throw NotSimple();
    target = std::min<uint64_t>(block_bytes, std::max<uint64_t>(1u << 20, p / i * block_records));
    std::vector<size_t> b{0};
    while (b.back() < len) b.push_back(len - b.back() <= target ? len : find_cut(data, len, b.back() + target));
    return b;
}

// Runs fn(i) for i < n on `threads` threads; rethrows the first exception.
template <class F>
void parallel_for(uint32_t threads, size_t n, F&& fn) {
    std::atomic<size_t> next{0};
    std::atomic<bool> stop{false};
    std::exception_ptr err;
    std::mutex mu;
    auto worker = [&] {
        try {
            for (size_t i; !stop && (i = next++) < n;) fn(i);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
            stop = true;
        }
    };
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < std::min<size_t>(threads, n); ++t) ts.emplace_back(worker);
    worker();
    for (auto& t : ts) t.join();
    if (err) std::rethrow_exception(err);
}

// Paired parallel cut (plain mapped files, GPU parsing): both files are cut at guessed record starts, the newlines
// of every block are counted in parallel (records per block = lines / 4), and each file-1 block is paired with the
// same record range of file 2, located by counting lines inside one file-2 block. The GPU checks every line group of
// both files, so any layout this does not fit fails there (or here) and the caller runs the sequential reader.
// Files with different record counts also go to the sequential reader (its zip rule and read-ahead decide).
StreamTotals run_paired_split(const std::shared_ptr<Buf>& m1, const std::shared_ptr<Buf>& m2, uint32_t threads,
                              Sink& sink, ShardSel shard, PackMode pm, int direct) {
    const uint64_t BLOCK_RECORDS = 1u << 15, BLOCK_BYTES = 12ull << 20;
    const char* d1 = m1->data();
    const char* d2 = m2->data();
    const std::vector<size_t> b1 = split_bounds(d1, m1->len, BLOCK_RECORDS, BLOCK_BYTES);
    const std::vector<size_t> b2 = split_bounds(d2, m2->len, BLOCK_RECORDS, BLOCK_BYTES);
    const size_t n1 = b1.size() - 1, n2 = b2.size() - 1;
    std::vector<uint64_t> recs(n1 + n2 + 2, 0);  // records per block, then exclusive sums per file
    parallel_for(threads, n1 + n2, [&](size_t i) {
        const bool f2 = i >= n1;
        const char* d = f2 ? d2 : d1;
        const std::vector<size_t>& b = f2 ? b2 : b1;
        const size_t j = f2 ? i - n1 : i, len = (f2 ? m2 : m1)->len;
        uint64_t lines = count_nl(d + b[j], b[j + 1] - b[j]);
        if (b[j + 1] == len && d[len - 1] != '\n') ++lines;
        if (lines == 0 || lines % 4 != 0) throw NotSimple();
        recs[i] = lines / 4;
    });
    std::vector<uint64_t> r1(n1 + 1, 0), r2(n2 + 1, 0);
    for (size_t j = 0; j < n1; ++j) r1[j + 1] = r1[j] + recs[j];
    for (size_t j = 0; j < n2; ++j) r2[j + 1] = r2[j] + recs[n1 + j];
    if (r1[n1] != r2[n2]) throw NotSimple();
    auto offset2 = [&](uint64_t r) -> size_t {  // byte offset of record r of file 2
        const size_t j = (size_t)(std::upper_bound(r2.begin(), r2.end(), r) - r2.begin()) - 1;
        if (j >= n2) return m2->len;
        if (r == r2[j]) return b2[j];
        return b2[j] + skip_lines(d2 + b2[j], b2[j + 1] - b2[j], 4 * (r - r2[j]));
    };
    std::atomic<uint64_t> batches{0}, records{0}, bases{0};
    parallel_for(threads, n1, [&](size_t i) {
        if (!shard.mine(i)) return;
        const size_t s2 = offset2(r1[i]), e2 = offset2(r1[i + 1]);
        const uint64_t l1 = b1[i + 1] - b1[i], l2 = e2 - s2, n = r1[i + 1] - r1[i];
        speq_slot s;
        if (pm.kind) {  // packed on the host: both files' records, mates interleaved
            sink.acquire(s, l1 + l2, 2 * n);
            uint64_t nb = 0;
            bool ok = false;
            try {
                ok = pack_records(d1, b1[i], b1[i + 1], m1->len, d2, s2, e2, m2->len, n, true, pm, s, l1 + l2, nb);
            } catch (...) {
                sink.submit(s, 0);
                throw;
            }
            if (!ok) {
                sink.submit(s, 0);
                throw NotSimple();
            }
            sink.submit_packed(s, 2 * n, pm.kind == 2);
            batches += 1;
            records += 2 * n;
            bases += nb;
            return;
        }
        sink.acquire_raw(s, l1 + l2);
        if (direct) {  // H2D straight from the mappings (the record counts came from the newline pass above)
            sink.submit_raw(s, l1, l2, n, true, d1 + b1[i], d2 + s2);
        } else {
            // copies with streaming stores where the destination is 16-B aligned (no read-for-ownership)
            (void)copy_count_nl(reinterpret_cast<char*>(s.seq), d1 + b1[i], l1);
            (void)copy_count_nl(reinterpret_cast<char*>(s.seq) + l1, d2 + s2, l2);
            sink.submit_raw(s, l1, l2, n, true);
        }
        batches += 1;
        records += 2 * n;
    });
    return {records.load(), bases.load(), batches.load()};
}

// Reader thread (cutting blocks of both files in step) + n_parsers parser threads feeding `sink`. With `split`, a
// mapped single-end file is cut at guessed record starts (find_cut, no per-record work on the reader) and each
// parser checks that its block is a chain of four-line records from its first byte to its last; since block 0
// starts at byte 0, the chains join into exactly the records the sequential cutter finds. Throws NotSimple when a
// block is not such a chain (the caller discards what was submitted and runs again without `split`).
StreamTotals run_stream(const char* path1, const char* path2, uint32_t threads, Sink& sink, bool gpu_parse,
                        bool split, ShardSel shard = {}, PackMode pm = {}, int direct = 0) {
    const bool paired = path2 != nullptr;
    const uint32_t n_parsers = std::max<uint32_t>(1, std::min<uint32_t>(threads ? threads : 1, 64));
    const uint64_t BLOCK_RECORDS = 1u << 15, BLOCK_BYTES = 12ull << 20;  // pipeline slots hold SLOT_BYTES
    // opened here so that a missing file fails before any thread starts
    const bool try_split = split && (!paired || gpu_parse);
    Cutter c1(path1, threads, !try_split);
    std::unique_ptr<Cutter> c2;
    if (paired) c2 = std::make_unique<Cutter>(path2, threads, !try_split);
    // direct 2: the mappings are page-locked (one registration each) and copied by DMA straight from the page
    // cache; every copy completes before they are released (drain, which runs before the cutters go)
    auto reg = [&](const std::shared_ptr<Buf>& m) {
        if (direct == 2 && m && !m->registered && m->map) m->registered = speq::host_register_readonly(m->map, m->map_len);
    };
    struct Drain {
        Sink& s;
        bool on;
        ~Drain() {
            if (on) try { s.drain_copies(); } catch (...) {}
        }
    } drain{sink, direct != 0};
    if (try_split && paired) {
        std::shared_ptr<Buf> m1 = c1.mapping(), m2 = c2->mapping();
        reg(m1);
        reg(m2);
        if (m1 && m2) return run_paired_split(m1, m2, n_parsers, sink, shard, pm, direct);
    }
    Shared sh;
    sh.max_q = n_parsers + 1;
    const std::shared_ptr<Buf> map = split && !paired ? c1.mapping() : nullptr;
    if (gpu_parse) reg(map);
    auto push = [&](Work&& w) {
        std::unique_lock<std::mutex> lk(sh.mu);
        sh.cv_put.wait(lk, [&] { return sh.q.size() < sh.max_q || sh.failed; });
        if (sh.failed) return false;
        sh.q.push_back(std::move(w));
        sh.cv_get.notify_one();
        return true;
    };
    auto split_reader = [&] {
        const char* data = map->data();
        const size_t len = map->len;
        // block bytes for about BLOCK_RECORDS records, from the first records' mean size
        uint64_t target = BLOCK_BYTES;
        {
            size_t p = 0, end = 0, sl = 0;
            uint32_t i = 0;
            for (; i < 256 && fast_record(data, len, p, true, end, sl); ++i) p = end;
            if (i == 0) throw NotSimple();
            target = std::min<uint64_t>(BLOCK_BYTES, std::max<uint64_t>(1u << 20, p / i * BLOCK_RECORDS));
        }
        for (size_t pos = 0, b = 0; pos < len; ++b) {
            const size_t e = len - pos <= target ? len : find_cut(data, len, pos + target);
            Work w;
            w.b1 = Block{map, pos, e, 0, true, 0};
            w.split = true;
            w.seq = b;
            if (shard.mine(b) && !push(std::move(w))) return;
            pos = e;
        }
    };
    auto reader = [&] {
        try {
            if (map) {
                split_reader();
                std::lock_guard<std::mutex> lk(sh.mu);
                sh.done = true;
                sh.cv_get.notify_all();
                return;
            }
            for (uint64_t b = 0;; ++b) {
                Work w;
                w.b1 = c1.next(BLOCK_RECORDS, BLOCK_BYTES);
                w.n = w.b1.n;
                if (paired && w.n) {
                    w.b2 = c2->next(w.n, ~0ull);
                    w.n = std::min(w.n, w.b2.n);  // views::zip stops at the shorter file
                }
                const bool last = w.n == 0 || (paired && w.b2.n < w.b1.n);
                w.seq = b;
                if (w.n && shard.mine(b) && !push(std::move(w))) return;
                if (last) break;
            }
            std::lock_guard<std::mutex> lk(sh.mu);
            sh.done = true;
            sh.cv_get.notify_all();
        } catch (const NotSimple& e) {
            sh.fail(e.what(), false, true);
        } catch (const IoError& e) {
            sh.fail(e.what(), true);
        } catch (const std::exception& e) {
            sh.fail(e.what(), false);
        }
    };
    auto parser = [&] {
        try {
            for (;;) {
                Work w;
                {
                    std::unique_lock<std::mutex> lk(sh.mu);
                    sh.cv_get.wait(lk, [&] { return !sh.q.empty() || sh.done; });
                    if (sh.failed || sh.q.empty()) return;
                    w = std::move(sh.q.front());
                    sh.q.pop_front();
                    sh.cv_put.notify_one();
                }
                if (w.split && pm.kind) {
                    // packed on the host: the record count from the newlines, then record by record (any record the
                    // four-line packer cannot take makes the caller run the sequential cutter instead)
                    const uint64_t l1 = w.b1.size();
                    const bool eof = w.b1.end == w.b1.buf->len;
                    uint64_t lines = count_nl(w.b1.data(), l1);
                    if (eof && l1 && w.b1.data()[l1 - 1] != '\n') ++lines;
                    if (lines == 0 || lines % 4 != 0) throw NotSimple();
                    speq_slot s;
                    sink.acquire(s, l1, lines / 4);
                    uint64_t nb = 0;
                    bool ok = false;
                    try {
                        ok = pack_records(w.b1.buf->data(), w.b1.begin, w.b1.end, w.b1.buf->len, nullptr, 0, 0, 0,
                                          lines / 4, false, pm, s, l1, nb);
                    } catch (...) {
                        sink.submit(s, 0);
                        throw;
                    }
                    if (!ok) {
                        sink.submit(s, 0);
                        throw NotSimple();
                    }
                    sink.submit_packed(s, lines / 4, pm.kind == 2);
                    sh.records += lines / 4;
                    sh.bases += nb;
                    sh.batches += 1;
                    if (sh.failed) return;
                    continue;
                }
                if (w.split && gpu_parse) {
                    // raw text to HBM; the record count comes from the newlines counted during the copy, and the
                    // GPU checks every line group (a failure makes the caller run the sequential cutter instead)
                    const uint64_t l1 = w.b1.size();
                    const bool eof = w.b1.end == w.b1.buf->len;
                    speq_slot s;
                    sink.acquire_raw(s, l1);
                    // direct: one read-only newline pass over the mapping, then H2D from the mapping itself — only
                    // for blocks of a whole-file mapping, which outlives every copy (run_stream drains them before
                    // the cutters go); a block of a recycled read / inflate buffer is always copied into the slot
                    const bool dir = direct != 0 && w.b1.buf && w.b1.buf->map != nullptr;
                    uint64_t lines = dir ? count_nl(w.b1.data(), l1)
                                         : copy_count_nl(reinterpret_cast<char*>(s.seq), w.b1.data(), l1);
                    if (eof && l1 && w.b1.data()[l1 - 1] != '\n') ++lines;
                    if (lines == 0 || lines % 4 != 0) {
                        sink.submit(s, 0);
                        throw NotSimple();
                    }
                    sink.submit_raw(s, l1, 0, lines / 4, false, dir ? w.b1.data() : nullptr);
                    sh.records += lines / 4;
                    sh.batches += 1;
                    if (sh.failed) return;
                    continue;
                }
                if (w.split) {
                    const char* base = w.b1.buf->data();
                    const bool eof = w.b1.end == w.b1.buf->len;
                    size_t p = w.b1.begin, end = 0, sl = 0;
                    uint64_t n = 0, bases = 0;
                    for (; p < w.b1.end; ++n, bases += sl, p = end)
                        if (!fast_record(base, w.b1.end, p, eof, end, sl)) throw NotSimple();
                    w.b1.n = w.n = n;
                    w.b1.bases = bases;
                }
                speq_slot s;
                const uint64_t recs = paired ? 2 * w.n : w.n;
                if (pm.kind && w.b1.simple && w.n == w.b1.n && (!paired || (w.b2.simple && w.n == w.b2.n))) {
                    // four-line records: packed on the host (falls through to the host parser when a record holds
                    // blanks or digits the grammar drops)
                    const uint64_t l1 = w.b1.size(), l2 = w.b2.size();
                    sink.acquire(s, l1 + l2, recs);
                    uint64_t nb = 0;
                    bool ok = false;
                    try {
                        ok = pack_records(w.b1.buf->data(), w.b1.begin, w.b1.end, w.b1.buf->len,
                                          paired ? w.b2.buf->data() : nullptr, w.b2.begin, w.b2.end,
                                          paired ? w.b2.buf->len : 0, w.n, paired, pm, s, l1 + l2, nb);
                    } catch (...) {
                        sink.submit(s, 0);
                        throw;
                    }
                    if (ok) {
                        sink.submit_packed(s, recs, pm.kind == 2);
                        sh.records += recs;
                        sh.bases += nb;
                        sh.batches += 1;
                        if (sh.failed) return;
                        continue;
                    }
                    sink.submit(s, 0);
                }
                if (gpu_parse && w.b1.simple && w.n == w.b1.n && (!paired || (w.b2.simple && w.n == w.b2.n))) {
                    // raw four-line text straight to HBM; records are split on the GPU (fastq_gpu.hip)
                    const uint64_t l1 = w.b1.size(), l2 = w.b2.size();
                    sink.acquire_raw(s, l1 + l2);
                    std::memcpy(s.seq, w.b1.data(), l1);
                    if (paired) std::memcpy(s.seq + l1, w.b2.data(), l2);
                    sink.submit_raw(s, l1, l2, w.n, paired);
                    sh.records += recs;  // bases: counted on the GPU (pipeline_gpu_parsed_bases)
                    sh.batches += 1;
                    if (sh.failed) return;
                    continue;
                }
                sink.acquire(s, w.b1.size() + w.b2.size(), recs);
                uint64_t out = 0;
                size_t p1 = 0, p2 = 0;
                s.offsets[0] = 0;
                try {
                    for (uint64_t i = 0; i < w.n; ++i) {
                        out = parse_record(w.b1.data(), w.b1.size(), p1, s.seq, s.qual, out, path1);
                        if (paired) {
                            s.offsets[2 * i + 1] = out;
                            out = parse_record(w.b2.data(), w.b2.size(), p2, s.seq, s.qual, out, path2);
                            s.offsets[2 * i + 2] = out;
                        } else {
                            s.offsets[i + 1] = out;
                        }
                    }
                    // the general grammar must end exactly where the cutter did
                    if ((w.n == w.b1.n && p1 != w.b1.size()) || (paired && p2 != w.b2.size()))
                        throw IoError(std::string("irregular FASTQ record layout in ") +
                                      (p1 != w.b1.size() ? path1 : path2));
                } catch (...) {
                    sink.submit(s, 0);
                    throw;
                }
                sink.submit(s, recs);
                sh.records += recs;
                sh.bases += out;
                sh.batches += 1;
                if (sh.failed) return;
            }
        } catch (const NotSimple& e) {
            sh.fail(e.what(), false, true);
        } catch (const IoError& e) {
            sh.fail(e.what(), true);
        } catch (const std::exception& e) {
            sh.fail(e.what(), false);
        }
    };
    std::vector<std::thread> ts;
    ts.emplace_back(reader);
    for (uint32_t i = 0; i < n_parsers; ++i) ts.emplace_back(parser);
    for (auto& t : ts) t.join();
    if (sh.failed) {
        if (sh.retry) throw NotSimple();
        if (sh.io_error) throw IoError(sh.error);
        throw speq::DeviceError(sh.error);
    }
    return {sh.records.load(), sh.bases.load(), sh.batches.load()};
}

// SPEQ_SPLIT_CUT=0 keeps the sequential cutter for single-end mapped files (A/B measurements).
bool split_cut_enabled() {
    const char* e = std::getenv("SPEQ_SPLIT_CUT");
    return !(e && e[0] == '0');
}


// The FASTQ scan over n >= 1 replicas of one index (one per GPU of this process): blocks are dealt to the replicas'
// pipelines in turn and each replica's counters accumulate on its own device; the sums over replicas are taken on
// the host at the end (G + 2 words per replica; the EM histograms are merged by speq_em_merge).
// shard / cut: speq_scan_fastq_shard (one process per GPU); the defaults are the single-process behaviour.
void scan_fastq_impl(speq_device_index* const* ds, speq_em* const* ems, uint32_t n_dev, const char* path1,
                     const char* path2, const speq_scan_params* params, uint32_t threads, uint64_t* counts,
                     double* weights, speq_stream_stats* stats, ShardSel shard = {}, int cut = -1) {
    if (!ds || n_dev == 0 || !path1 || !params || !counts) throw std::invalid_argument("speq_scan_fastq: null argument");
    if (params->mode == SPEQ_MODE_LOCAL && !weights)
        throw std::invalid_argument("speq_scan_fastq: local mode needs weights");
    const bool paired = path2 != nullptr;
    if ((params->paired != 0) != paired)
        throw std::invalid_argument("speq_scan_fastq: params->paired must match the presence of path2");
    for (uint32_t i = 0; i < n_dev; ++i)
        if (!ds[i] || speq::device_groups(ds[i]) != speq::device_groups(ds[0]) ||
            speq::device_text_len(ds[i]) != speq::device_text_len(ds[0]))
            throw std::invalid_argument("speq_scan_fastq_multi: replicas of different indexes");
    const uint32_t G = speq::device_groups(ds[0]);
    const auto t0 = std::chrono::steady_clock::now();
    // one replica: parsers + 2 slots (up to SPEQ_STREAM_SLOTS_MAX, default 18: 9.5 -> 8.6 ms at cfg 2 with 16 parsers,
    // profiles/r02/stream_slots.jsonl); several: the same total spread over
    // them, at least 3 each
    const uint32_t want = stream_slots(threads);
    const uint32_t n_slots = n_dev == 1 ? want : std::max<uint32_t>(3, (want + n_dev - 1) / n_dev + 1);
    std::vector<std::unique_ptr<speq_pipeline, void (*)(speq_pipeline*)>> guards;
    std::vector<speq_pipeline*> pls;
    for (uint32_t i = 0; i < n_dev; ++i) {
        guards.emplace_back(speq::acquire_cached_pipeline(ds[i], params, ems ? ems[i] : nullptr,
                                                          paired ? 2 * SLOT_BYTES : SLOT_BYTES,
                                                          paired ? 2u << 15 : 1u << 15, n_slots),
                            speq_pipeline_free);
        pls.push_back(guards.back().get());
    }
    PipelineSink sink(pls);
    bool gpu_parse = true;
    for (uint32_t i = 0; i < n_dev; ++i) gpu_parse = gpu_parse && speq::device_fastq_gpu(ds[i]);
    // SPEQ_FASTQ_PACK=1: four-line records packed on the host (3 bits per base in global mode, a byte in local mode)
    // instead of raw text parsed on the GPU. Off by default: at 16 host threads the packer (~180 ns per 150-bp record)
    // is slower than the PCIe transfer of the raw text it saves (cfg 2: 11.0 vs 9.9 ms, profiles/r02/stream_pack.jsonl)
    PackMode pm;
    {
        const char* fp = std::getenv("SPEQ_FASTQ_PACK");
        if (fp && fp[0] == '1') pm.kind = params->mode == SPEQ_MODE_GLOBAL ? 2 : 1;
        pm.cutoff = params->phred_cutoff;
    }
    // SPEQ_FASTQ_DIRECT (A/B knob, default 0 = copy into the pinned slots): raw blocks of a mapped file go to the GPU
    // straight from the page-cache mapping, the parsers only counting newlines — 1: hipMemcpyAsync from the pageable
    // mapping; 2: the mapping page-locked once (hipHostRegister, read-only) and copied by DMA.
    int direct = 0;
    {
        const char* e = std::getenv("SPEQ_FASTQ_DIRECT");
        if (e && (e[0] == '1' || e[0] == '2')) direct = e[0] - '0';
    }
    std::vector<uint64_t> scratch(SPEQ_COUNTS_LEN(G));
    std::vector<double> wscratch(std::max<uint32_t>(G, 1));
    auto attempt = [&](bool split) {
        try {
            StreamTotals t = run_stream(path1, path2, threads, sink, gpu_parse, split, shard, pm, direct);
            // split blocks are parsed on the GPU unchecked by the host: any failed check means a layout the
            // parallel cut cannot handle (or a malformed file) -> sequential run, which reports real errors
            if (split && gpu_parse) {
                uint32_t err = 0;
                for (speq_pipeline* pl : pls) err |= speq::pipeline_take_parse_errors(pl);
                if (err) throw NotSimple();
            }
            return t;
        } catch (...) {  // drain the pipelines and zero their counters
            for (speq_pipeline* pl : pls) (void)speq_pipeline_finish(pl, scratch.data(), wscratch.data());
            throw;
        }
    };
    StreamTotals tot;
    try {
        tot = attempt(cut < 0 ? split_cut_enabled() : cut == 1);
    } catch (const NotSimple&) {
        if (ems)
            for (uint32_t i = 0; i < n_dev; ++i) speq::em_clear(ems[i]);
        if (cut == 1) {  // the other ranks must agree before anyone runs the sequential cutter
            for (uint32_t i = 0; i < n_dev; ++i) speq::return_cached_pipeline(ds[i], guards[i].release());
            throw speq::RetryError("speq_scan_fastq_shard: the parallel cut does not fit this input");
        }
        tot = attempt(false);
    }
    std::fill(counts, counts + SPEQ_COUNTS_LEN(G), 0);
    if (weights) std::fill(weights, weights + G, 0.0);
    for (uint32_t i = 0; i < n_dev; ++i) {  // replica order: the fp64 weight sums are deterministic
        check_rc(speq_pipeline_finish(pls[i], scratch.data(), wscratch.data()));
        for (size_t j = 0; j < scratch.size(); ++j) counts[j] += scratch[j];
        if (weights && params->mode == SPEQ_MODE_LOCAL)
            for (uint32_t g = 0; g < G; ++g) weights[g] += wscratch[g];
        tot.bases += speq::pipeline_gpu_parsed_bases(pls[i]);
    }
    for (uint32_t i = 0; i < n_dev; ++i) speq::return_cached_pipeline(ds[i], guards[i].release());
    if (stats) {
        stats->records = tot.records;
        stats->bases = tot.bases;
        stats->batches = tot.batches;
        stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
}

}  // namespace

extern "C" int speq_stream_reserve(int device, uint32_t threads, uint32_t paired) {
    return speq::guarded([&] {
        if (device < 0) throw std::invalid_argument("speq_stream_reserve: bad device ordinal");
        speq::reserve_slot_buffers(device, stream_slots(threads), paired ? 2 * SLOT_BYTES : SLOT_BYTES,
                                   paired ? 2u << 15 : 1u << 15, paired != 0);
    });
}

extern "C" int speq_scan_fastq(speq_device_index* d, const char* path1, const char* path2,
                               const speq_scan_params* params, speq_em* em, uint32_t threads, uint64_t* counts,
                               double* weights, speq_stream_stats* stats) {
    return speq::guarded([&] {
        speq_em* ems[1] = {em};
        scan_fastq_impl(&d, em ? ems : nullptr, 1, path1, path2, params, threads, counts, weights, stats);
    });
}

extern "C" int speq_scan_fastq_multi(speq_device_index* const* ds, speq_em* const* ems, uint32_t n_devices,
                                     const char* path1, const char* path2, const speq_scan_params* params,
                                     uint32_t threads, uint64_t* counts, double* weights, speq_stream_stats* stats) {
    return speq::guarded([&] {
        scan_fastq_impl(ds, ems, n_devices, path1, path2, params, threads, counts, weights, stats);
    });
}

extern "C" int speq_scan_fastq_shard(speq_device_index* d, speq_em* em, const char* path1, const char* path2,
                                     const speq_scan_params* params, uint32_t threads, uint32_t shard,
                                     uint32_t n_shards, int cut, uint64_t* counts, double* weights,
                                     speq_stream_stats* stats) {
    return speq::guarded([&] {
        if (n_shards == 0 || shard >= n_shards) throw std::invalid_argument("speq_scan_fastq_shard: bad shard");
        if (cut < -1 || cut > 1) throw std::invalid_argument("speq_scan_fastq_shard: cut must be -1, 0 or 1");
        if (cut == -1 && n_shards > 1)
            throw std::invalid_argument("speq_scan_fastq_shard: several shards need cut 0 or 1 (ranks must agree)");
        speq_em* ems[1] = {em};
        scan_fastq_impl(&d, em ? ems : nullptr, 1, path1, path2, params, threads, counts, weights, stats,
                        ShardSel{shard, n_shards}, cut);
    });
}

extern "C" int speq_fastq_checksum_shard(const char* path1, const char* path2, uint32_t threads, uint32_t shard,
                                         uint32_t n_shards, int cut, uint64_t* records, uint64_t* bases,
                                         uint64_t* digest) {
    return speq::guarded([&] {
        if (!path1 || !records || !bases || !digest) throw std::invalid_argument("speq_fastq_checksum_shard: null argument");
        if (n_shards == 0 || shard >= n_shards) throw std::invalid_argument("speq_fastq_checksum_shard: bad shard");
        if (cut != 0 && cut != 1) throw std::invalid_argument("speq_fastq_checksum_shard: cut must be 0 or 1");
        auto sink = std::make_unique<ChecksumSink>();
        StreamTotals tot;
        try {
            tot = run_stream(path1, path2, threads, *sink, false, cut == 1, ShardSel{shard, n_shards});
        } catch (const NotSimple&) {
            throw speq::RetryError("speq_fastq_checksum_shard: the parallel cut does not fit this input");
        }
        *records = tot.records;
        *bases = tot.bases;
        *digest = sink->digest.load();
    });
}

extern "C" int speq_fastq_checksum(const char* path1, const char* path2, uint32_t threads, uint64_t* records,
                                   uint64_t* bases, uint64_t* digest) {
    return speq::guarded([&] {
        if (!path1 || !records || !bases || !digest) throw std::invalid_argument("speq_fastq_checksum: null argument");
        auto sink = std::make_unique<ChecksumSink>();
        StreamTotals tot;
        try {
            tot = run_stream(path1, path2, threads, *sink, false, split_cut_enabled());
        } catch (const NotSimple&) {
            sink = std::make_unique<ChecksumSink>();
            tot = run_stream(path1, path2, threads, *sink, false, false);
        }
        *records = tot.records;
        *bases = tot.bases;
        *digest = sink->digest.load();
    });
}
