// Times the first use of each of libspeq_scan.so's code objects (HIP loads a translation unit's code object at the
// first use of one of its kernels), one after the other, after the runtime has started. Built by `make probes`;
// run on the GPU box: tools/module_load_probe [lib path] [order: letters a s f b]
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

int main(int argc, char** argv) {
    const char* lib = argc > 1 ? argv[1] : "speq_amd/libspeq_scan.so";
    const char* order = argc > 2 ? argv[2] : "asfb";
    using clk = std::chrono::steady_clock;
    // SPEQ_PROBE_PRELOAD=1: the library is loaded before the runtime starts (as in `speq`, which links it)
    const bool pre = std::getenv("SPEQ_PROBE_PRELOAD") != nullptr;
    void* h = pre ? dlopen(lib, RTLD_NOW) : nullptr;
    auto t0 = clk::now();
    if (hipFree(nullptr) != hipSuccess) return 1;
    auto t1 = clk::now();
    std::printf("runtime start %.1f ms (library %s)\n", std::chrono::duration<double, std::milli>(t1 - t0).count(),
                pre ? "loaded before" : "not loaded");
    if (!h) h = dlopen(lib, RTLD_NOW);
    if (!h) {
        std::printf("dlopen: %s\n", dlerror());
        return 1;
    }
    for (const char* c = order; *c; ++c) {
        const char* sym = *c == 'a'   ? "_ZN4speq19warm_module_ax_scanEv"
                          : *c == 's' ? "_ZN4speq24warm_module_scan_kernelsEv"
                          : *c == 'f' ? "_ZN4speq21warm_module_fastq_gpuEv"
                                      : "_ZN4speq21warm_module_build_gpuEv";
        auto fn = reinterpret_cast<void (*)()>(dlsym(h, sym));
        if (!fn) {
            std::printf("missing %s\n", sym);
            return 1;
        }
        auto a = clk::now();
        fn();
        auto b = clk::now();
        std::printf("%s %.1f ms\n", sym, std::chrono::duration<double, std::milli>(b - a).count());
    }
    return 0;
}
