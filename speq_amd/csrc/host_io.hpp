// Host-side input layer (reference L3): groupings parser and FASTA/FASTQ readers.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace speq {

// speq::file_to_map, /root/reference/src/file_to_map.cpp:20-119, same line grammar and error messages:
//   Name(count): i, j-k, …    ('#' starts a comment; lines without ':' are ignored; later lines win;
//                               gaps are -1; "(count)" is mandatory and a line without it throws).
struct Groupings {
    std::vector<std::string> names;
    std::vector<int> scaffolds;  // record index -> group index (-1 unassigned)
    std::vector<int> counts;
};
// Throws IoError when the file cannot be opened (the reference silently yields empty groupings there;
// DESIGN.md documents the difference) and std::invalid_argument for a missing/non-numeric "(count)"
// (std::stoi at file_to_map.cpp:43). Parse errors inside a token list go to `err` like std::cerr.
Groupings parse_groupings(const std::string& path, std::string* err);
Groupings parse_groupings_text(const std::string& text, std::string* err);

// Sequence records as one concatenated byte buffer + offsets (n + 1 entries).
struct SeqBatch {
    std::vector<char> seq;
    std::vector<char> qual;      // empty for FASTA
    std::vector<uint64_t> offsets{0};
    std::vector<std::string> ids;
    bool has_qual = false;
    uint64_t size() const { return offsets.size() - 1; }
};

// Reads a whole FASTA or FASTQ file (format detected from the first record marker).
SeqBatch read_sequences(const std::string& path, bool keep_ids);

// Streaming FASTQ reader for large read files (reads up to `max_records` records per call).
class FastqReader {
public:
    explicit FastqReader(const std::string& path);
    ~FastqReader();
    // Appends up to max_records records to `out` (which must be empty); returns the number read.
    uint64_t next(SeqBatch& out, uint64_t max_records, uint64_t max_bytes);
    bool eof() const { return eof_; }
private:
    bool getline(std::string& line);
    void* fp_ = nullptr;
    std::string path_;
    std::string pending_;
    bool has_pending_ = false;
    bool eof_ = false;
};

// seqan3 debug_stream formatting of a vector: "[a,b,c]" with default ostream formatting of each element.
std::string format_vector(const std::vector<double>& v);
std::string format_vector(const std::vector<uint64_t>& v);

}  // namespace speq
