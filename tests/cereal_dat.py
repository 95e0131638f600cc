"""Test helper: the reference's `<stem>_<k>mer.dat` bytes, restated from cereal's published binary encoding.

The reference writes `oarchive(index_file_time); oarchive(unique_kmers); oarchive(total_kmers);` through a
`cereal::BinaryOutputArchive` (/root/reference/src/fm_scanner.cpp:1561-1571) and reads it back the same way
(:91-119). cereal is an un-vendored dependency of the reference (upstream cereal 1.3.x). Its binary
archive writes, in native (little-endian) byte order:
  * std::chrono::time_point -> its duration -> the duration's `count()` as the raw rep (cereal/types/chrono.hpp);
    `std::filesystem::file_time_type` is libstdc++'s `__file_clock` time point: int64 nanoseconds since the
    file-clock epoch, which is the system epoch + 6437664000 s (checked against `last_write_time` with this image's g++);
  * std::vector<size_t> -> a size tag of cereal's `size_type` (uint64) and then the elements as one binary block
    (cereal/types/vector.hpp, arithmetic-element overload).
"""
import struct

FILE_CLOCK_EPOCH_DIFF_NS = 6437664000 * 10**9


def file_time_ns(st_mtime_ns):
    """`last_write_time(p).time_since_epoch().count()` for a file whose `st_mtime_ns` is given."""
    return st_mtime_ns - FILE_CLOCK_EPOCH_DIFF_NS


def encode(stamp_ns, unique, total):
    out = struct.pack("<q", stamp_ns)
    for v in (unique, total):
        out += struct.pack("<Q", len(v)) + struct.pack(f"<{len(v)}Q", *v)
    return out


def decode(data):
    (stamp,) = struct.unpack_from("<q", data, 0)
    off, vecs = 8, []
    for _ in range(2):
        (n,) = struct.unpack_from("<Q", data, off)
        vecs.append(list(struct.unpack_from(f"<{n}Q", data, off + 8)))
        off += 8 + 8 * n
    assert off == len(data), "trailing bytes"
    return stamp, vecs[0], vecs[1]
