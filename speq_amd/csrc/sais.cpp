// SA-IS, induced sorting of LMS substrings with one level of recursion per reduced string.
// See sais.hpp for the contract.
#include "sais.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace speq {
namespace {

// Bucket heads (end=false) or one-past-tails (end=true) for every symbol.
template <typename T>
void bucket_bounds(const T* s, int64_t n, int32_t K, std::vector<int64_t>& bkt, bool end) {
    std::fill(bkt.begin(), bkt.end(), 0);
    for (int64_t i = 0; i < n; ++i) bkt[s[i]]++;
    int64_t sum = 0;
    for (int32_t c = 0; c < K; ++c) {
        sum += bkt[c];
        bkt[c] = end ? sum : sum - bkt[c];
    }
}

struct TypeVec {  // 1 = S-type, 0 = L-type
    std::vector<uint8_t> t;
    bool s(int64_t i) const { return t[i] != 0; }
    bool lms(int64_t i) const { return i > 0 && t[i] && !t[i - 1]; }
};

template <typename T>
void induce(const T* s, int32_t* sa, int64_t n, int32_t K, const TypeVec& tv, std::vector<int64_t>& bkt) {
    // L-type suffixes, left to right from bucket heads.
    bucket_bounds(s, n, K, bkt, false);
    for (int64_t i = 0; i < n; ++i) {
        int64_t j = (int64_t)sa[i] - 1;
        if (sa[i] > 0 && !tv.s(j)) sa[bkt[s[j]]++] = (int32_t)j;
    }
    // S-type suffixes, right to left from bucket tails.
    bucket_bounds(s, n, K, bkt, true);
    for (int64_t i = n - 1; i >= 0; --i) {
        int64_t j = (int64_t)sa[i] - 1;
        if (sa[i] > 0 && tv.s(j)) sa[--bkt[s[j]]] = (int32_t)j;
    }
}

template <typename T>
void sais_rec(const T* s, int32_t* sa, int64_t n, int32_t K) {
    if (n == 1) { sa[0] = 0; return; }
    TypeVec tv;
    tv.t.assign(n, 0);
    tv.t[n - 1] = 1;
    for (int64_t i = n - 2; i >= 0; --i)
        tv.t[i] = (s[i] < s[i + 1] || (s[i] == s[i + 1] && tv.t[i + 1])) ? 1 : 0;

    std::vector<int64_t> bkt(K);
    // Stage 1: place LMS suffixes at bucket tails and induce to sort the LMS substrings.
    bucket_bounds(s, n, K, bkt, true);
    std::fill(sa, sa + n, -1);
    for (int64_t i = 1; i < n; ++i)
        if (tv.lms(i)) sa[--bkt[s[i]]] = (int32_t)i;
    induce(s, sa, n, K, tv, bkt);

    // Compact the sorted LMS substrings into sa[0..n1).
    int64_t n1 = 0;
    for (int64_t i = 0; i < n; ++i)
        if (tv.lms(sa[i])) sa[n1++] = sa[i];

    // Name the LMS substrings; equal substrings share a name.
    std::fill(sa + n1, sa + n, -1);
    int32_t name = 0;
    int64_t prev = -1;
    for (int64_t i = 0; i < n1; ++i) {
        int64_t pos = sa[i];
        bool diff = false;
        for (int64_t d = 0; d < n; ++d) {
            if (prev == -1 || s[pos + d] != s[prev + d] || tv.t[pos + d] != tv.t[prev + d]) {
                diff = true;
                break;
            }
            if (d > 0 && (tv.lms(pos + d) || tv.lms(prev + d))) break;
        }
        if (diff) { ++name; prev = pos; }
        sa[n1 + pos / 2] = name - 1;  // LMS positions are >= 2 apart
    }
    for (int64_t i = n - 1, j = n - 1; i >= n1; --i)
        if (sa[i] >= 0) sa[j--] = sa[i];

    // Stage 2: sort the reduced string (recursively if names are not unique).
    int32_t* s1 = sa + n - n1;
    int32_t* sa1 = sa;
    if (name < n1) {
        sais_rec<int32_t>(s1, sa1, n1, name);
    } else {
        for (int64_t i = 0; i < n1; ++i) sa1[s1[i]] = (int32_t)i;
    }

    // Stage 3: induce the full suffix array from the sorted LMS suffixes.
    bucket_bounds(s, n, K, bkt, true);
    for (int64_t i = 1, j = 0; i < n; ++i)
        if (tv.lms(i)) s1[j++] = (int32_t)i;
    for (int64_t i = 0; i < n1; ++i) sa1[i] = s1[sa1[i]];
    std::fill(sa + n1, sa + n, -1);
    for (int64_t i = n1 - 1; i >= 0; --i) {
        int64_t j = sa[i];
        sa[i] = -1;
        sa[--bkt[s[j]]] = (int32_t)j;
    }
    induce(s, sa, n, K, tv, bkt);
}

}  // namespace

void sais_u8(const uint8_t* s, int32_t* sa, int64_t n, int32_t alphabet) {
    if (n < 1 || n >= (int64_t(1) << 31)) throw std::invalid_argument("sais: text length out of range");
    if (s[n - 1] != 0) throw std::invalid_argument("sais: text must end with the unique symbol 0");
    for (int64_t i = 0; i + 1 < n; ++i)
        if (s[i] == 0 || s[i] >= alphabet) throw std::invalid_argument("sais: bad symbol in text");
    sais_rec<uint8_t>(s, sa, n, alphabet);
}

}  // namespace speq
