// Does the HIP runtime carve small hipMallocs out of a larger block (GPU_MAX_SUBALLOC_SIZE)?
// For each size: 4 allocations, their pointers, hipMemGetAddressRange's base / size (the
// block the runtime really allocated) and whether hipIpcGetMemHandle accepts them.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/suballoc_probe.cpp -o tools/bin/suballoc_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

int main() {
    const size_t KiB = 1024, MiB = 1024 * KiB;
    const size_t sizes[] = {64 * KiB, 1 * MiB, 2 * MiB - 4 * KiB, 2 * MiB, 2 * MiB + 4 * KiB, 4 * MiB, 6 * MiB, 8 * MiB, 16 * MiB};
    const char *env = getenv("GPU_MAX_SUBALLOC_SIZE");
    printf("{\"GPU_MAX_SUBALLOC_SIZE\": \"%s\"}\n", env ? env : "(unset)");
    for (size_t sz : sizes) {
        for (int i = 0; i < 4; ++i) {
            void *p = nullptr;
            if (hipMalloc(&p, sz) != hipSuccess) { printf("{\"size\": %zu, \"error\": \"hipMalloc\"}\n", sz); return 1; }
            hipDeviceptr_t base = nullptr;
            size_t range = 0;
            const hipError_t er = hipMemGetAddressRange(&base, &range, reinterpret_cast<hipDeviceptr_t>(p));
            hipIpcMemHandle_t h;
            const hipError_t ei = hipIpcGetMemHandle(&h, p);
            (void)hipGetLastError();
            printf("{\"size\": %zu, \"i\": %d, \"ptr\": \"%p\", \"range_rc\": %d, \"base\": \"%p\", \"range\": %zu, "
                   "\"offset\": %lld, \"ipc_rc\": %d}\n", sz, i, p, int(er), (void *)base, range,
                   (long long)(static_cast<char *>(p) - static_cast<char *>((void *)base)), int(ei));
        }
    }
    return 0;
}
