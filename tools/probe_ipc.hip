// probe_ipc.hip — which device allocations can hipIpcGetMemHandle export?
// Diagnostic only (tools/), not part of the library.
#include <hip/hip_runtime.h>

#include <cstdio>

static void probe(const char *what, void *p) {
    void *base = nullptr;
    size_t size = 0;
    hipError_t e1 = hipMemGetAddressRange(&base, &size, p);
    hipIpcMemHandle_t h;
    hipError_t e2 = hipIpcGetMemHandle(&h, base);
    hipError_t e3 = hipIpcGetMemHandle(&h, p);
    printf("%-40s p=%p base=%p size=%zu range=%s get(base)=%s get(p)=%s\n", what, p, base, size,
           hipGetErrorName(e1), hipGetErrorName(e2), hipGetErrorName(e3));
    (void)hipGetLastError();
}

int main() {
    void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
    hipMalloc(&a, 65536);
    probe("fresh 64KiB", a);
    hipMalloc(&b, size_t(256) << 20);
    probe("fresh 256MiB", b);
    hipFree(b);
    hipMalloc(&c, 65536);
    probe("64KiB after freeing 256MiB", c);
    hipMalloc(&d, size_t(2) << 20);
    probe("2MiB after freeing 256MiB", d);
    void *e[8];
    for (int i = 0; i < 8; ++i) {
        hipMalloc(&e[i], size_t(64) << 20);
    }
    for (int i = 0; i < 8; ++i) hipFree(e[i]);
    void *f = nullptr, *g = nullptr, *k = nullptr;
    hipMalloc(&f, 262144);
    probe("256KiB after freeing 8x64MiB", f);
    hipMalloc(&g, size_t(4) << 20);
    probe("4MiB after freeing 8x64MiB", g);
    hipMalloc(&k, size_t(64) << 20);
    probe("64MiB after freeing 8x64MiB", k);
    void *sm[4];
    for (int i = 0; i < 4; ++i) {
        hipMalloc(&sm[i], 4096);
        char name[64];
        snprintf(name, sizeof(name), "small 4KiB #%d", i);
        probe(name, sm[i]);
    }
    return 0;
}
