// Process teardown cost by what the process holds: allocates `vram_mb` of device memory in `nbuf` buffers and
// `pinned_mb` of registered host memory, prints the wall clock (ns since the epoch) and leaves with _Exit.
// tools/exit_probe.py runs it and measures the time from that print to the process's end.
// Usage: tools/build/exit_probe vram_mb pinned_mb nbuf [streams]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    const size_t vram = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 0) << 20;
    const size_t pinned = (argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 0) << 20;
    const int nbuf = argc > 3 ? std::atoi(argv[3]) : 1;
    const int nstreams = argc > 4 ? std::atoi(argv[4]) : 0;
    if (hipFree(nullptr) != hipSuccess) return 1;
    void* scratch = nullptr;
    if (hipMalloc(&scratch, 64) != hipSuccess) return 6;
    for (int i = 0; i < nstreams; ++i) {  // each stream bound to a hardware queue by a command
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 7;
        if (hipMemsetAsync(scratch, 0, 64, st) != hipSuccess) return 8;
    }
    for (int i = 0; i < nbuf && vram; ++i) {
        void* p = nullptr;
        if (hipMalloc(&p, vram / nbuf) != hipSuccess) return 2;
        if (hipMemset(p, 0, vram / nbuf) != hipSuccess) return 3;
    }
    if (pinned) {
        void* h = std::aligned_alloc(4096, pinned);
        std::memset(h, 0, pinned);
        if (hipHostRegister(h, pinned, hipHostRegisterDefault) != hipSuccess) return 4;
    }
    if (hipDeviceSynchronize() != hipSuccess) return 5;
    const long long t = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::system_clock::now().time_since_epoch()).count();
    std::printf("%lld\n", t);
    std::fflush(stdout);
    std::_Exit(0);
}
