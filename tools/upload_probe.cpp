// Host -> device upload of an index-sized pageable buffer, four ways, each on fresh host and device memory:
// plain hipMemcpy (the runtime stages pageable memory), hipHostRegister + hipMemcpy + unregister, copies through a
// ring of pinned staging buffers (memcpy into them by T threads, hipMemcpyAsync out), and the same plain hipMemcpy
// split over T threads. Run on the GPU box: tools/build/upload_probe [MiB] [threads]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#define OK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                    \
        }                                                                    \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 377;
    const int T = argc > 2 ? std::atoi(argv[2]) : 8;
    const size_t n = mib << 20;
    auto t0 = clk::now();
    OK(hipFree(nullptr));
    std::printf("runtime %.1f ms\n", ms(t0, clk::now()));
    if (argc > 3 && std::strcmp(argv[3], "d2h") == 0) {
        // the process's first device -> host copies of `mib` MiB into registered memory (after one host -> device
        // copy, as in a scan), three in a row
        std::vector<unsigned char> h(n);
        void* d = nullptr;
        OK(hipMalloc(&d, n));
        OK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
        for (int rep = 0; rep < 3; ++rep) {
            std::unique_ptr<unsigned char[]> o(new unsigned char[n]);
            auto a = clk::now();
            OK(hipHostRegister(o.get(), n, hipHostRegisterDefault));
            auto r = clk::now();
            OK(hipMemcpy(o.get(), d, n, hipMemcpyDeviceToHost));
            auto c = clk::now();
            OK(hipHostUnregister(o.get()));
            std::printf("d2h %d: register %.2f ms, copy %.2f ms\n", rep, ms(a, r), ms(r, c));
        }
        return 0;
    }
    if (argc > 3 && std::strcmp(argv[3], "first") == 0) {
        // the process's first host -> device copy, registered, of `mib` MiB; with argv[4] == "tiny", after one
        // 64-byte pageable copy (does the first copy pay a one-time set-up?)
        const bool tiny = argc > 4 && std::strcmp(argv[4], "tiny") == 0;
        std::vector<unsigned char> h(n);
        for (size_t i = 0; i < n; i += 4096) h[i] = (unsigned char)i;
        void* d = nullptr;
        OK(hipMalloc(&d, n));
        if (tiny) {
            auto a = clk::now();
            OK(hipMemcpy(d, h.data(), 64, hipMemcpyHostToDevice));
            std::printf("tiny pageable copy %.1f ms\n", ms(a, clk::now()));
        }
        for (int rep = 0; rep < 2; ++rep) {
            auto a = clk::now();
            OK(hipHostRegister(h.data(), n, hipHostRegisterDefault));
            auto r = clk::now();
            OK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
            auto c = clk::now();
            OK(hipHostUnregister(h.data()));
            std::printf("registered copy %d: register %.1f ms, copy %.1f ms (%.1f GB/s)\n", rep, ms(a, r), ms(r, c),
                        n / 1e6 / ms(r, c));
        }
        return 0;
    }
    if (argc > 3 && std::strcmp(argv[3], "alloc") == 0) {
        // pinned host memory of `mib` MiB in T threads (one buffer each): hipHostMalloc, or an aligned allocation
        // touched and then registered
        for (int form = 0; form < 2; ++form) {
            std::vector<void*> bufs(T, nullptr);
            const size_t each = n / T;
            auto a = clk::now();
            std::vector<std::thread> ts;
            for (int t = 0; t < T; ++t)
                ts.emplace_back([&, t] {
                    if (form == 0) {
                        OK(hipHostMalloc(&bufs[t], each, hipHostMallocDefault));
                    } else {
                        bufs[t] = std::aligned_alloc(4096, each);
                        std::memset(bufs[t], 0, each);
                        OK(hipHostRegister(bufs[t], each, hipHostRegisterDefault));
                    }
                });
            for (auto& x : ts) x.join();
            auto b = clk::now();
            for (int t = 0; t < T; ++t) {
                if (form == 0) {
                    OK(hipHostFree(bufs[t]));
                } else {
                    OK(hipHostUnregister(bufs[t]));
                    std::free(bufs[t]);
                }
            }
            std::printf("%s: %.1f ms to allocate, %.1f ms to free\n", form ? "aligned_alloc + touch + register" : "hipHostMalloc",
                        ms(a, b), ms(b, clk::now()));
        }
        return 0;
    }
    for (int form = 0; form < 4; ++form) {
        std::vector<unsigned char> h(n);
        for (size_t i = 0; i < n; i += 4096) h[i] = (unsigned char)i;  // touched, like a loaded index
        void* d = nullptr;
        OK(hipMalloc(&d, n));
        auto a = clk::now();
        if (form == 0) {
            OK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
        } else if (form == 1) {
            OK(hipHostRegister(h.data(), n, hipHostRegisterDefault));
            auto r = clk::now();
            OK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
            auto c = clk::now();
            OK(hipHostUnregister(h.data()));
            std::printf("  register %.1f ms, copy %.1f ms, unregister %.1f ms\n", ms(a, r), ms(r, c), ms(c, clk::now()));
        } else if (form == 2) {
            const size_t piece = 8u << 20;
            const int ring = 2 * T;
            std::vector<void*> st(ring);
            std::vector<hipEvent_t> ev(ring);
            std::vector<hipStream_t> ss(T);
            for (int i = 0; i < ring; ++i) {
                OK(hipHostMalloc(&st[i], piece, hipHostMallocDefault));
                OK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
            }
            for (int t = 0; t < T; ++t) OK(hipStreamCreateWithFlags(&ss[t], hipStreamNonBlocking));
            auto p = clk::now();
            std::vector<std::thread> ts;
            const size_t pieces = (n + piece - 1) / piece;
            for (int t = 0; t < T; ++t)
                ts.emplace_back([&, t] {
                    int use = 0;
                    for (size_t q = t; q < pieces; q += T, ++use) {
                        const int slot = 2 * t + (use & 1);
                        OK(hipEventSynchronize(ev[slot]));
                        const size_t off = q * piece, len = n - off < piece ? n - off : piece;
                        std::memcpy(st[slot], h.data() + off, len);
                        OK(hipMemcpyAsync(static_cast<unsigned char*>(d) + off, st[slot], len, hipMemcpyHostToDevice,
                                          ss[t]));
                        OK(hipEventRecord(ev[slot], ss[t]));
                    }
                    OK(hipStreamSynchronize(ss[t]));
                });
            for (auto& x : ts) x.join();
            std::printf("  pinned ring: allocation %.1f ms, copies %.1f ms\n", ms(a, p), ms(p, clk::now()));
            for (int i = 0; i < ring; ++i) {
                OK(hipHostFree(st[i]));
                OK(hipEventDestroy(ev[i]));
            }
            for (int t = 0; t < T; ++t) OK(hipStreamDestroy(ss[t]));
        } else {
            std::vector<std::thread> ts;
            for (int t = 0; t < T; ++t)
                ts.emplace_back([&, t] {
                    const size_t a0 = n * t / T, a1 = n * (t + 1) / T;
                    OK(hipMemcpy(static_cast<unsigned char*>(d) + a0, h.data() + a0, a1 - a0, hipMemcpyHostToDevice));
                });
            for (auto& x : ts) x.join();
        }
        const char* names[4] = {"pageable hipMemcpy", "registered", "pinned ring", "pageable, threads"};
        std::printf("%-20s %.1f ms (%.1f GB/s)\n", names[form], ms(a, clk::now()), n / 1e6 / ms(a, clk::now()));
        OK(hipFree(d));
    }
    return 0;
}
