// SA-IS suffix-array construction (Nong, Zhang & Chan, "Two efficient algorithms for linear time suffix
// array construction", IEEE ToC 2011), written from the published algorithm.
//
// Replaces the SDSL suffix-array construction that seqan3::fm_index runs inside
// /root/reference/src/fm_indexer.cpp:36 (upstream, not vendored).
#pragma once
#include <cstdint>

namespace speq {

// Builds the suffix array of s[0..n) into sa[0..n).
// Requirements: n >= 1, s[n-1] == 0 and 0 occurs nowhere else, every symbol < alphabet.
// n must be < 2^31.
void sais_u8(const uint8_t* s, int32_t* sa, int64_t n, int32_t alphabet);

}  // namespace speq
