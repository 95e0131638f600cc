// Collectives of a one-process-per-GPU job: the end-of-scan counter exchange. Replaces the host future.get()
// reductions of per-thread vectors at /root/reference/src/fm_scanner.cpp:224-233 (and :497-505, :740-748,
// :1006-1022, :1550-1560). The message is G+2 u64 (<= 1.6 KB at G = 200): latency-bound, one call per scan.
//
// Two transports behind one handle (speq_comm):
//  * RCCL (ncclAllReduce over xGMI), the multi-GPU path: one rank per GPU;
//  * host sockets (loopback TCP, a reduce at rank 0 in rank order and a broadcast), chosen by speq_comm_connect when
//    ranks share a GPU (RCCL refuses two ranks on one device) or when asked for; the sums are the same.
// speq_comm_connect does the rendezvous itself: rank 0 listens on 127.0.0.1 and publishes {nonce, port} in a file;
// the other ranks connect and present the nonce (a stale file of a dead run is ignored: its port refuses, or its
// nonce does not match), and rank 0 hands out the RCCL id over the sockets when RCCL is chosen.
//
// librccl (~570 MB with its device code) is loaded on first use with dlopen, not linked: a single-GPU `speq scan`
// or Python process never maps it (linking it cost every process start the load and registration of its code).
#include <arpa/inet.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "capi_internal.hpp"
#include "em.hpp"
#include "scan_internal.hpp"

namespace {
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::string failure;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = ::dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = ::dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = ::dlerror();
            failure = std::string("cannot load librccl.so.1: ") + (e ? e : "unknown error");
            return;
        }
        auto sym = [&](const char* name) {
            void* f = ::dlsym(h, name);
            if (!f && failure.empty()) failure = std::string("librccl.so.1 lacks ") + name;
            return f;
        };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    });
    if (!failure.empty()) throw speq::DeviceError(failure);
    return r;
}

void nccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw speq::DeviceError(std::string(what) + ": " + rccl().error_string(r));
}

// ---- sockets ----
void send_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) throw speq::DeviceError(std::string("speq comm: send failed: ") + std::strerror(errno));
        c += w;
        n -= (size_t)w;
    }
}
void recv_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
        const ssize_t r = ::recv(fd, c, n, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r == 0) throw speq::DeviceError("speq comm: a peer closed its connection");
        if (r < 0) throw speq::DeviceError(std::string("speq comm: recv failed: ") + std::strerror(errno));
        c += r;
        n -= (size_t)r;
    }
}
void send_u64(int fd, uint64_t v) { send_all(fd, &v, 8); }
uint64_t recv_u64(int fd) {
    uint64_t v = 0;
    recv_all(fd, &v, 8);
    return v;
}
void set_nodelay(int fd) {
    int one = 1;
    (void)::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
}  // namespace

// The handle behind every `void* comm` of the C ABI.
struct speq_comm {
    int transport = SPEQ_COMM_RCCL;
    int nranks = 1, rank = 0;
    ncclComm_t nccl = nullptr;
    std::vector<int> fds;  // rank 0: fds[r] = socket to rank r (fds[0] unused); others: fds[0] = socket to rank 0
    ~speq_comm() {
        for (int fd : fds)
            if (fd >= 0) ::close(fd);
    }
};

namespace {
speq_comm* as_comm(void* c) {
    if (!c) throw std::invalid_argument("speq comm: null communicator");
    return static_cast<speq_comm*>(c);
}

constexpr uint64_t RDZV_MAGIC = 0x5350455152445A31ull;  // "SPEQRDZ1"
constexpr uint64_t HELLO_MAGIC = 0x5350455148454C4Full;  // "SPEQHELO"

std::string bus_id(int device) {
    if (device < 0) return std::string();
    char id[64] = {0};
    if (hipDeviceGetPCIBusId(id, (int)sizeof(id), device) != hipSuccess)
        throw speq::DeviceError("speq_comm_connect: cannot query GPU " + std::to_string(device));
    return std::string(id);
}

// In-place reduction over the ranks of a host-socket communicator: rank 0 receives every other rank's buffer in
// rank order, combines, and sends the result back (deterministic: the same order as a sequential loop over ranks).
template <typename T, typename Op>
void host_allreduce(speq_comm* c, T* buf, uint64_t count, Op op) {
    if (c->nranks == 1 || count == 0) return;
    const size_t bytes = (size_t)count * sizeof(T);
    if (c->rank == 0) {
        std::vector<T> tmp(count);
        for (int r = 1; r < c->nranks; ++r) {
            recv_all(c->fds[r], tmp.data(), bytes);
            for (uint64_t i = 0; i < count; ++i) buf[i] = op(buf[i], tmp[i]);
        }
        for (int r = 1; r < c->nranks; ++r) send_all(c->fds[r], buf, bytes);
    } else {
        send_all(c->fds[0], buf, bytes);
        recv_all(c->fds[0], buf, bytes);
    }
}
}  // namespace

extern "C" {

int speq_comm_unique_id(void* id_out) {
    return speq::guarded([&] {
        if (!id_out) throw std::invalid_argument("speq_comm_unique_id: null argument");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
        ncclUniqueId id;
        nccl_ok(rccl().get_unique_id(&id), "ncclGetUniqueId");
        std::memcpy(id_out, &id, sizeof(id));
    });
}

int speq_comm_init(int nranks, int rank, const void* id, void** comm_out) {
    return speq::guarded([&] {
        if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks)
            throw std::invalid_argument("speq_comm_init: bad argument");
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        auto c = std::make_unique<speq_comm>();
        c->nranks = nranks;
        c->rank = rank;
        c->transport = SPEQ_COMM_RCCL;
        nccl_ok(rccl().comm_init_rank(&c->nccl, nranks, uid, rank), "ncclCommInitRank");
        *comm_out = c.release();
    });
}

int speq_comm_connect(int nranks, int rank, int device, const char* rendezvous_path, int transport, int timeout_s,
                      void** comm_out) {
    return speq::guarded([&] {
        if (!comm_out || !rendezvous_path || !*rendezvous_path || nranks < 1 || rank < 0 || rank >= nranks ||
            transport < SPEQ_COMM_AUTO || transport > SPEQ_COMM_HOST)
            throw std::invalid_argument("speq_comm_connect: bad argument");
        if (transport != SPEQ_COMM_HOST && device < 0)
            throw std::invalid_argument("speq_comm_connect: RCCL needs a GPU (device >= 0)");
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s > 0 ? timeout_s : 600);
        auto expired = [&] { return std::chrono::steady_clock::now() > deadline; };
        const std::string path(rendezvous_path);
        const std::string my_bus = transport == SPEQ_COMM_HOST ? std::string() : bus_id(device);
        auto c = std::make_unique<speq_comm>();
        c->nranks = nranks;
        c->rank = rank;
        c->fds.assign(rank == 0 ? nranks : 1, -1);
        int chosen = SPEQ_COMM_HOST;
        unsigned char uid[128] = {0};
        if (rank == 0) {
            const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
            if (ls < 0) throw speq::DeviceError("speq_comm_connect: socket() failed");
            struct Closer {
                int fd;
                ~Closer() { ::close(fd); }
            } lclose{ls};
            sockaddr_in addr{};
            addr.sin_family = AF_INET;
            addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
            addr.sin_port = 0;
            if (::bind(ls, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(ls, nranks) != 0)
                throw speq::DeviceError(std::string("speq_comm_connect: cannot listen on 127.0.0.1: ") +
                                        std::strerror(errno));
            socklen_t alen = sizeof(addr);
            ::getsockname(ls, reinterpret_cast<sockaddr*>(&addr), &alen);
            const uint64_t nonce = std::random_device{}() ^ ((uint64_t)std::random_device{}() << 32) ^
                                   (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
            {  // publish {magic, nonce, port} atomically, readable by this user only (the nonce is the credential)
                const std::string tmp = path + ".tmp." + std::to_string((long)::getpid());
                (void)::unlink(tmp.c_str());
                const int tfd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0600);
                const uint64_t rec[3] = {RDZV_MAGIC, nonce, (uint64_t)ntohs(addr.sin_port)};
                bool ok_w = tfd >= 0 && ::write(tfd, rec, sizeof(rec)) == (ssize_t)sizeof(rec);
                if (tfd >= 0) ok_w = (::close(tfd) == 0) && ok_w;
                if (!ok_w || std::rename(tmp.c_str(), path.c_str()) != 0) {
                    (void)::unlink(tmp.c_str());
                    throw speq::DeviceError("speq_comm_connect: cannot write the rendezvous file " + path);
                }
            }
            std::vector<std::string> buses(nranks);
            buses[0] = my_bus;
            int joined = 1;
            while (joined < nranks) {
                pollfd pf{ls, POLLIN, 0};
                const int pr = ::poll(&pf, 1, 200);
                if (expired())
                    throw speq::DeviceError("speq_comm_connect: " + std::to_string(nranks - joined) +
                                            " rank(s) did not join within the timeout");
                if (pr <= 0) continue;
                const int fd = ::accept(ls, nullptr, nullptr);
                if (fd < 0) continue;
                try {  // hello: {magic, nonce, rank, bus id length, bus id}
                    timeval tv{10, 0};
                    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
                    const uint64_t m = recv_u64(fd), nn = recv_u64(fd), r = recv_u64(fd), bl = recv_u64(fd);
                    if (m != HELLO_MAGIC || nn != nonce || r == 0 || r >= (uint64_t)nranks || bl > 64 ||
                        c->fds[r] >= 0)
                        throw speq::DeviceError("bad hello");
                    std::string b(bl, '\0');
                    if (bl) recv_all(fd, &b[0], bl);
                    timeval none{0, 0};
                    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
                    set_nodelay(fd);
                    c->fds[r] = fd;
                    buses[r] = b;
                    ++joined;
                } catch (const std::exception&) {
                    ::close(fd);
                }
            }
            if (transport == SPEQ_COMM_AUTO) {
                std::vector<std::string> s(buses);
                std::sort(s.begin(), s.end());
                const bool distinct = std::adjacent_find(s.begin(), s.end()) == s.end();
                chosen = (distinct && nranks > 1) ? SPEQ_COMM_RCCL : SPEQ_COMM_HOST;
                if (nranks == 1) chosen = SPEQ_COMM_RCCL;
            } else {
                chosen = transport;
            }
            if (chosen == SPEQ_COMM_RCCL) {
                ncclUniqueId id;
                nccl_ok(rccl().get_unique_id(&id), "ncclGetUniqueId");
                std::memcpy(uid, &id, sizeof(uid));
            }
            for (int r = 1; r < nranks; ++r) {
                send_u64(c->fds[r], (uint64_t)chosen);
                send_all(c->fds[r], uid, sizeof(uid));
            }
        } else {
            for (;;) {
                if (expired())
                    throw speq::DeviceError("speq_comm_connect: rank " + std::to_string(rank) +
                                            " found no live rendezvous at " + path);
                uint64_t rec[3] = {0, 0, 0};
                {
                    std::ifstream is(path, std::ios::binary);
                    if (!is.read(reinterpret_cast<char*>(rec), sizeof(rec)) || rec[0] != RDZV_MAGIC) {
                        std::this_thread::sleep_for(std::chrono::milliseconds(20));
                        continue;
                    }
                }
                const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
                if (fd < 0) throw speq::DeviceError("speq_comm_connect: socket() failed");
                sockaddr_in addr{};
                addr.sin_family = AF_INET;
                addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
                addr.sin_port = htons((uint16_t)rec[2]);
                if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
                    ::close(fd);  // a stale file (its listener is gone), or rank 0 not listening yet
                    std::this_thread::sleep_for(std::chrono::milliseconds(50));
                    continue;
                }
                try {
                    // rank 0's reply must arrive before the deadline too (a listener that never answers)
                    const auto left = std::chrono::duration_cast<std::chrono::microseconds>(
                        deadline - std::chrono::steady_clock::now()).count();
                    timeval tv{(time_t)(std::max<long long>(left, 1000) / 1000000),
                               (suseconds_t)(std::max<long long>(left, 1000) % 1000000)};
                    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
                    send_u64(fd, HELLO_MAGIC);
                    send_u64(fd, rec[1]);
                    send_u64(fd, (uint64_t)rank);
                    send_u64(fd, (uint64_t)my_bus.size());
                    if (!my_bus.empty()) send_all(fd, my_bus.data(), my_bus.size());
                    set_nodelay(fd);
                    chosen = (int)recv_u64(fd);  // a listener of another run closes on our nonce: retry
                    recv_all(fd, uid, sizeof(uid));
                    timeval none{0, 0};
                    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
                } catch (const std::exception&) {
                    ::close(fd);
                    std::this_thread::sleep_for(std::chrono::milliseconds(50));
                    continue;
                }
                c->fds[0] = fd;
                break;
            }
        }
        c->transport = chosen;
        if (rank == 0) std::remove(path.c_str());  // every rank has joined: the file has served its purpose
        if (chosen == SPEQ_COMM_RCCL) {
            int prev = 0;
            if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
                throw speq::DeviceError("speq_comm_connect: cannot select GPU " + std::to_string(device));
            struct Restore {
                int dev;
                ~Restore() { (void)hipSetDevice(dev); }
            } restore{prev};
            ncclUniqueId id;
            std::memcpy(&id, uid, sizeof(id));
            nccl_ok(rccl().comm_init_rank(&c->nccl, nranks, id, rank), "ncclCommInitRank");
        }
        *comm_out = c.release();
    });
}

int speq_comm_transport(void* comm) {
    if (!comm) return SPEQ_E_ARG;
    return static_cast<speq_comm*>(comm)->transport;
}

int speq_comm_destroy(void* comm) {
    return speq::guarded([&] {
        if (!comm) return;
        std::unique_ptr<speq_comm> c(static_cast<speq_comm*>(comm));
        if (c->nccl) nccl_ok(rccl().comm_destroy(c->nccl), "ncclCommDestroy");
    });
}

int speq_allreduce_u64(void* comm, uint64_t* d_buf, uint64_t count, void* stream) {
    return speq::guarded([&] {
        speq_comm* c = as_comm(comm);
        if (!d_buf) throw std::invalid_argument("speq_allreduce_u64: null argument");
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (c->transport == SPEQ_COMM_RCCL) {
            nccl_ok(rccl().all_reduce(d_buf, d_buf, count, ncclUint64, ncclSum, c->nccl, st), "ncclAllReduce");
            return;
        }
        std::vector<uint64_t> h(count);
        if (hipMemcpyAsync(h.data(), d_buf, count * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_u64: copy to the host failed");
        host_allreduce(c, h.data(), count, [](uint64_t a, uint64_t b) { return a + b; });
        if (hipMemcpyAsync(d_buf, h.data(), count * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_u64: copy to the device failed");
    });
}

int speq_allreduce_f64(void* comm, double* d_buf, uint64_t count, void* stream) {
    return speq::guarded([&] {
        speq_comm* c = as_comm(comm);
        if (!d_buf) throw std::invalid_argument("speq_allreduce_f64: null argument");
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (c->transport == SPEQ_COMM_RCCL) {
            nccl_ok(rccl().all_reduce(d_buf, d_buf, count, ncclFloat64, ncclSum, c->nccl, st), "ncclAllReduce");
            return;
        }
        std::vector<double> h(count);
        if (hipMemcpyAsync(h.data(), d_buf, count * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_f64: copy to the host failed");
        host_allreduce(c, h.data(), count, [](double a, double b) { return a + b; });
        if (hipMemcpyAsync(d_buf, h.data(), count * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_f64: copy to the device failed");
    });
}

int speq_allreduce_host(void* comm, int device, void* buf, uint64_t count, int is_f64) {
    return speq::guarded([&] {
        speq_comm* c = as_comm(comm);
        if (!buf && count) throw std::invalid_argument("speq_allreduce_host: null argument");
        if (count == 0) return;
        if (c->transport == SPEQ_COMM_HOST) {
            if (is_f64) host_allreduce(c, static_cast<double*>(buf), count, [](double a, double b) { return a + b; });
            else host_allreduce(c, static_cast<uint64_t*>(buf), count, [](uint64_t a, uint64_t b) { return a + b; });
            return;
        }
        int prev = 0;
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_host: cannot select GPU " + std::to_string(device));
        void* d = nullptr;
        struct Release {
            int dev;
            void*& p;
            ~Release() {
                if (p) (void)hipFree(p);
                (void)hipSetDevice(dev);
            }
        } release{prev, d};
        const size_t bytes = (size_t)count * 8;
        if (hipMalloc(&d, bytes) != hipSuccess) throw speq::DeviceError("speq_allreduce_host: hipMalloc failed");
        if (hipMemcpy(d, buf, bytes, hipMemcpyHostToDevice) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_host: copy to the device failed");
        nccl_ok(rccl().all_reduce(d, d, count, is_f64 ? ncclFloat64 : ncclUint64, ncclSum, c->nccl, nullptr),
                "ncclAllReduce");
        if (hipMemcpy(buf, d, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_host: copy to the host failed");
    });
}

int speq_em_allreduce(speq_em* em, void* comm, void* stream) {
    return speq::guarded([&] {
        speq_comm* c = as_comm(comm);
        if (!em) throw std::invalid_argument("speq_em_allreduce: null argument");
        if (em->finalized || !em->d_mult) throw std::invalid_argument("speq_em_allreduce: histogram already finalized");
        int prev = 0;
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(speq::device_ordinal(em->dev)) != hipSuccess)
            throw speq::DeviceError("speq_em_allreduce: cannot select the histogram's GPU");
        struct Restore {
            int dev;
            ~Restore() { (void)hipSetDevice(dev); }
        } restore{prev};
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (c->transport == SPEQ_COMM_RCCL) {
            // interval ends are 0 wherever a rank never wrote (speq_em_create / em_clear zero them), so the max is
            // the interval end wherever any rank saw the interval start
            nccl_ok(rccl().all_reduce(em->d_mult, em->d_mult, em->n, ncclUint32, ncclSum, c->nccl, st),
                    "ncclAllReduce");
            nccl_ok(rccl().all_reduce(em->d_hi, em->d_hi, em->n, ncclUint32, ncclMax, c->nccl, st), "ncclAllReduce");
            if (hipStreamSynchronize(st) != hipSuccess) throw speq::DeviceError("speq_em_allreduce: stream failed");
            return;
        }
        // host sockets: the nonzero positions travel as {position, multiplicity, interval end} triples
        if (hipStreamSynchronize(st) != hipSuccess) throw speq::DeviceError("speq_em_allreduce: stream failed");
        std::vector<uint32_t> mult(em->n), hi(em->n);
        if (hipMemcpy(mult.data(), em->d_mult, em->n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(hi.data(), em->d_hi, em->n * 4, hipMemcpyDeviceToHost) != hipSuccess)
            throw speq::DeviceError("speq_em_allreduce: copy to the host failed");
        if (c->nranks > 1) {
            auto pack = [&] {
                std::vector<uint32_t> t;
                for (uint64_t i = 0; i < em->n; ++i)
                    if (mult[i]) {
                        t.push_back((uint32_t)i);
                        t.push_back(mult[i]);
                        t.push_back(hi[i]);
                    }
                return t;
            };
            auto send_vec = [&](int fd, const std::vector<uint32_t>& v) {
                send_u64(fd, v.size());
                if (!v.empty()) send_all(fd, v.data(), v.size() * 4);
            };
            auto recv_vec = [&](int fd) {  // {position, multiplicity, end} triples, at most one per position
                const uint64_t len = recv_u64(fd);
                if (len % 3 != 0 || len > 3 * em->n)
                    throw speq::DeviceError("speq_em_allreduce: a peer sent a malformed histogram length");
                std::vector<uint32_t> v(len);
                if (!v.empty()) recv_all(fd, v.data(), v.size() * 4);
                return v;
            };
            if (c->rank == 0) {
                for (int r = 1; r < c->nranks; ++r) {
                    const std::vector<uint32_t> t = recv_vec(c->fds[r]);
                    for (size_t i = 0; i + 2 < t.size(); i += 3) {
                        if (t[i] >= em->n) throw speq::DeviceError("speq_em_allreduce: a peer sent a bad position");
                        mult[t[i]] += t[i + 1];
                        hi[t[i]] = std::max(hi[t[i]], t[i + 2]);
                    }
                }
                const std::vector<uint32_t> all = pack();
                for (int r = 1; r < c->nranks; ++r) send_vec(c->fds[r], all);
            } else {
                send_vec(c->fds[0], pack());
                const std::vector<uint32_t> all = recv_vec(c->fds[0]);
                std::fill(mult.begin(), mult.end(), 0u);
                std::fill(hi.begin(), hi.end(), 0u);
                for (size_t i = 0; i + 2 < all.size(); i += 3) {
                    if (all[i] >= em->n) throw speq::DeviceError("speq_em_allreduce: rank 0 sent a bad position");
                    mult[all[i]] = all[i + 1];
                    hi[all[i]] = all[i + 2];
                }
            }
        }
        if (hipMemcpy(em->d_mult, mult.data(), em->n * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(em->d_hi, hi.data(), em->n * 4, hipMemcpyHostToDevice) != hipSuccess)
            throw speq::DeviceError("speq_em_allreduce: copy to the device failed");
    });
}

}  // extern "C"
