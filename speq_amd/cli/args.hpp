// Command line of `speq [index|scan|all] [options]`.
// Mirrors speq::args (/root/reference/include/arg_parse.h:10-37, src/arg_parse.cpp:3-203): the same
// sub-commands, option letters/names and defaults. seqan3::argument_parser is replaced by a small parser.
#pragma once
#include <cstdint>
#include <filesystem>
#include <stdexcept>
#include <string>
#include <vector>

namespace speq::args {

struct CmdArguments {  // include/arg_parse.h:10-28
    std::filesystem::path in_file_reads_path_1{};
    std::filesystem::path in_file_reads_path_2{};
    std::filesystem::path in_file_references{};
    std::filesystem::path in_file_references_groups{};
    std::filesystem::path io_file_index{"output.idx"};
    std::filesystem::path out_file_path{"output.txt"};
    bool is_force{};
    unsigned int threads{2};
    unsigned int kmer{70};
    unsigned int phred_cutoff{30};
    double fixed_accuracy{0.0};
    double precision{1e-6};
    bool is_indexer{false};
    bool is_scanner{false};
    bool is_parsed{false};
    // MI355X build extensions (not in the reference)
    unsigned int prefix_q{12};   // --prefix-q: q-mer interval table of the FM-index (levels q, q-1, q-2)
    bool pair_steps{true};       // --pair-steps: two-symbol occ planes
    unsigned triple_steps{2};    // --triple-steps: three-symbol occ planes (2 = auto)
    int gpu_build{-1};           // --gpu-build: -1 auto (GPU when one is visible), 0 host SA-IS, 1 GPU
    unsigned label_table{2};     // --label-table: per-position {group, run distance} table (2 = auto)
    int device{-1};              // --device: GPU ordinal (default: $LOCAL_RANK or 0)
    int gpus{1};                 // --gpus: scan on GPUs 0..N-1 of this process (0 = every visible GPU)
    std::vector<int> devices;    // --devices: explicit GPU ordinals (repeats = logical shards of one GPU)
    unsigned int max_em_iterations{1000};
};

struct ParseError : std::runtime_error {
    explicit ParseError(const std::string& m) : std::runtime_error(m) {}
};

// Parses argv; prints help and returns is_parsed=false for -h/--help; throws ParseError on bad input
// (the reference prints "speq <sub> | argument parsing error: …", src/arg_parse.cpp:41-45).
CmdArguments parse(int argc, char** argv);

// src/arg_parse.cpp:167-202
void check_in_file(std::filesystem::path& p);
void check_out_file(std::filesystem::path& p, bool is_force);

}  // namespace speq::args
