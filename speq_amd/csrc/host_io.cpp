// Groupings parser, FASTA/FASTQ readers and debug_stream-style vector formatting.
#include "host_io.hpp"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "capi_internal.hpp"
#include "speq_errors.hpp"

namespace speq {
namespace {

// utils::string_strip (file_to_map.cpp:3-8): removes tabs and spaces anywhere in the token.
std::string strip_blanks(std::string s) {
    s.erase(std::remove_if(s.begin(), s.end(), [](char c) { return c == '\t' || c == ' '; }), s.end());
    return s;
}

// utils::is_integer (file_to_map.cpp:10-18): optional sign or digit first, strtol must consume it all.
bool whole_integer(const std::string& s) {
    if (s.empty()) return false;
    const unsigned char c0 = (unsigned char)s[0];
    if (!std::isdigit(c0) && c0 != '-' && c0 != '+') return false;
    char* end = nullptr;
    std::strtol(s.c_str(), &end, 10);
    return *end == '\0';
}

constexpr long MAX_RECORD_INDEX = 1L << 28;

int record_index(const std::string& s) {
    const long v = std::atol(s.c_str());
    if (v < 0 || v >= MAX_RECORD_INDEX)
        throw std::invalid_argument("groupings: record index out of range: " + s);
    return (int)v;
}

void assign(std::vector<int>& scaffolds, int first, int last, int group) {
    if ((size_t)last + 1 > scaffolds.size()) scaffolds.resize((size_t)last + 1, -1);
    for (int i = first; i <= last; ++i) scaffolds[(size_t)i] = group;
}

}  // namespace

Groupings parse_groupings_text(const std::string& text, std::string* err) {
    Groupings g;
    std::istringstream in(text);
    std::string line;
    int group = -1;
    std::ostringstream errs;
    while (std::getline(in, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (line.find(':') == std::string::npos) continue;
        // "Name(count): …" — same index arithmetic as file_to_map.cpp:37-42, including npos wrap-around
        // (a line without "(count)" hands the whole line to std::stoi, which throws).
        const size_t open = line.find('(');
        g.names.push_back(line.substr(0, open));
        const size_t close = line.find(')');
        const std::string count_text = line.substr(open + 1, close - open - 1);
        try {
            g.counts.push_back(std::stoi(count_text));
        } catch (const std::exception&) {
            throw std::invalid_argument("groupings: missing or non-numeric \"(count)\" in line: " + line);
        }
        ++group;
        std::stringstream tokens(line.substr(line.find(':') + 1));
        std::string tok;
        while (std::getline(tokens, tok, ',')) {
            const size_t hy = tok.find('-');
            if (hy != std::string::npos) {
                const std::string a = strip_blanks(tok.substr(0, hy));
                const std::string b = strip_blanks(tok.substr(hy + 1));
                if (whole_integer(a) && whole_integer(b)) {
                    assign(g.scaffolds, record_index(a), record_index(b), group);
                } else {
                    errs << "Error in parsing groupings line: " << line
                         << "\nA non-integer range was detected and ignored at: " << strip_blanks(tok) << "\n";
                }
            } else {
                const std::string t = strip_blanks(tok);
                if (whole_integer(t)) {
                    const int i = record_index(t);
                    assign(g.scaffolds, i, i, group);
                } else {
                    errs << "Error in parsing groupings line: " << line
                         << "\nA non-integer index was detected and ignored at: " << t << "\n";
                }
            }
        }
    }
    if (err) *err = errs.str();
    return g;
}

Groupings parse_groupings(const std::string& path, std::string* err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw IoError("cannot open groupings file " + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return parse_groupings_text(ss.str(), err);
}

// ---------------------------------------------------------------------------------------------------
namespace {

inline bool is_seq_char(unsigned char c) { return !std::isspace(c) && !std::isdigit(c); }

void append_clean(std::vector<char>& dst, const std::string& line) {
    for (unsigned char c : line)
        if (is_seq_char(c)) dst.push_back((char)c);
}

}  // namespace

SeqBatch read_sequences(const std::string& path, bool keep_ids) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw IoError("cannot open sequence file " + path);
    SeqBatch b;
    std::string line;
    // skip leading empty lines
    while (std::getline(f, line) && line.find_first_not_of(" \t\r") == std::string::npos) {}
    if (!f && line.empty()) return b;
    if (line[0] == '>') {
        do {
            if (!line.empty() && line[0] == '>') {
                if (b.ids.size() > b.size()) b.offsets.push_back(b.seq.size());
                std::string id = line.substr(1);
                if (!id.empty() && id.back() == '\r') id.pop_back();
                b.ids.push_back(keep_ids ? id : std::string());
            } else if (!line.empty() && line[0] != ';') {
                if (b.ids.empty()) throw IoError("FASTA sequence before the first header in " + path);
                append_clean(b.seq, line);
            }
        } while (std::getline(f, line));
        if (b.ids.size() > b.size()) b.offsets.push_back(b.seq.size());
        if (!keep_ids) b.ids.clear();
        return b;
    }
    if (line[0] != '@') throw IoError("unrecognised sequence file format (expected FASTA '>' or FASTQ '@'): " + path);
    f.close();
    FastqReader r(path);
    r.next(b, ~0ull, ~0ull);
    if (!keep_ids) b.ids.clear();
    return b;
}

FastqReader::FastqReader(const std::string& path) : path_(path) {
    fp_ = std::fopen(path.c_str(), "rb");
    if (!fp_) throw IoError("cannot open reads file " + path);
}

FastqReader::~FastqReader() {
    if (fp_) std::fclose(static_cast<FILE*>(fp_));
}

bool FastqReader::getline(std::string& line) {
    if (has_pending_) {
        line.swap(pending_);
        has_pending_ = false;
        return true;
    }
    char* buf = nullptr;
    size_t cap = 0;
    ssize_t n = ::getline(&buf, &cap, static_cast<FILE*>(fp_));
    if (n < 0) {
        std::free(buf);
        eof_ = true;
        return false;
    }
    while (n > 0 && (buf[n - 1] == '\n' || buf[n - 1] == '\r')) --n;
    line.assign(buf, (size_t)n);
    std::free(buf);
    return true;
}

uint64_t FastqReader::next(SeqBatch& out, uint64_t max_records, uint64_t max_bytes) {
    out.has_qual = true;
    uint64_t got = 0;
    std::string line, seq, qual;
    while (got < max_records && (out.seq.size() < max_bytes || got == 0)) {
        // header
        bool found = false;
        while (getline(line)) {
            if (line.empty()) continue;
            if (line[0] != '@') {
                if (line[0] == '>') throw IoError("reads must be FASTQ (qualities are required): " + path_);
                throw IoError("malformed FASTQ record header in " + path_ + ": " + line);
            }
            found = true;
            break;
        }
        if (!found) break;
        out.ids.push_back(line.substr(1));
        seq.clear();
        qual.clear();
        bool plus = false;
        while (getline(line)) {
            if (!line.empty() && line[0] == '+') { plus = true; break; }
            for (unsigned char c : line)
                if (is_seq_char(c)) seq.push_back((char)c);
        }
        if (!plus) throw IoError("truncated FASTQ record (no '+' line) in " + path_);
        while (qual.size() < seq.size() && getline(line)) {
            for (unsigned char c : line)
                if (!std::isspace(c)) qual.push_back((char)c);
        }
        if (qual.size() != seq.size())
            throw IoError("FASTQ record with sequence/quality length mismatch in " + path_);
        out.seq.insert(out.seq.end(), seq.begin(), seq.end());
        out.qual.insert(out.qual.end(), qual.begin(), qual.end());
        out.offsets.push_back(out.seq.size());
        ++got;
    }
    return got;
}

std::string format_vector(const std::vector<double>& v) {
    std::ostringstream os;
    os << '[';
    for (size_t i = 0; i < v.size(); ++i) os << (i ? "," : "") << v[i];
    os << ']';
    return os.str();
}

std::string format_vector(const std::vector<uint64_t>& v) {
    std::ostringstream os;
    os << '[';
    for (size_t i = 0; i < v.size(); ++i) os << (i ? "," : "") << v[i];
    os << ']';
    return os.str();
}

}  // namespace speq

// ---- C ABI: groupings (so tests can check the parser without the CLI) ----
struct speq_groupings {
    speq::Groupings g;
    std::string err;
};

extern "C" {

int speq_groupings_parse(const char* path, speq_groupings** out) {
    return speq::guarded([&] {
        if (!path || !out) throw std::invalid_argument("speq_groupings_parse: null argument");
        auto* h = new speq_groupings();
        try {
            h->g = speq::parse_groupings(path, &h->err);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}
uint32_t speq_groupings_n_groups(const speq_groupings* g) { return g ? (uint32_t)g->g.names.size() : 0; }
const char* speq_groupings_name(const speq_groupings* g, uint32_t i) {
    return (g && i < g->g.names.size()) ? g->g.names[i].c_str() : nullptr;
}
int32_t speq_groupings_count(const speq_groupings* g, uint32_t i) {
    return (g && i < g->g.counts.size()) ? g->g.counts[i] : 0;
}
uint32_t speq_groupings_n_entries(const speq_groupings* g) { return g ? (uint32_t)g->g.scaffolds.size() : 0; }
const int32_t* speq_groupings_scaffolds(const speq_groupings* g) {
    return (g && !g->g.scaffolds.empty()) ? g->g.scaffolds.data() : nullptr;
}
const char* speq_groupings_errors(const speq_groupings* g) { return g ? g->err.c_str() : ""; }
void speq_groupings_free(speq_groupings* g) { delete g; }

}  // extern "C"
