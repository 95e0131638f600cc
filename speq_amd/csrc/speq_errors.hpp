// Exception types mapped onto the C ABI status codes (speq_scan.h). The C++ CLI catches them and prints
// to stderr the way the reference's uncaught exceptions surface (failure detection).
#pragma once
#include <stdexcept>
#include <string>

namespace speq {

struct IoError : std::runtime_error {
    explicit IoError(const std::string& m) : std::runtime_error(m) {}
};
struct GroupsError : std::runtime_error {
    explicit GroupsError(const std::string& m) : std::runtime_error(m) {}
};
struct DeviceError : std::runtime_error {
    explicit DeviceError(const std::string& m) : std::runtime_error(m) {}
};
// the parallel FASTQ cut does not fit the file (SPEQ_E_RETRY): the caller runs the sequential cutter on every rank
struct RetryError : std::runtime_error {
    explicit RetryError(const std::string& m) : std::runtime_error(m) {}
};

}  // namespace speq
