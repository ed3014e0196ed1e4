// probe_flags.hip — can two processes' GPUs synchronise through flags in a shared,
// host-registered /dev/shm page, and what does one signal+wait kernel cost?
// Diagnostic only (tools/), not part of the library.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void k_sync(unsigned *flags, int rank, int world, unsigned value, long long timeout,
                       unsigned *err) {
    if (threadIdx.x != 0) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(&flags[rank], value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long t0 = wall_clock64();
    for (int q = 0; q < world; ++q) {
        while (__hip_atomic_load(&flags[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
            if (wall_clock64() - t0 > timeout) {
                __hip_atomic_store(err, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

static int run(int rank, unsigned *host) {
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    hipError_t e = hipHostRegister(host, 4096, hipHostRegisterMapped);
    unsigned *dev = nullptr;
    hipError_t e2 = hipHostGetDevicePointer(reinterpret_cast<void **>(&dev), host, 0);
    printf("rank %d: wallclock %d kHz register=%s devptr=%s host=%p dev=%p\n", rank, khz,
           hipGetErrorName(e), hipGetErrorName(e2), (void *)host, (void *)dev);
    if (e != hipSuccess || e2 != hipSuccess) return 1;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const long long timeout = (long long)khz * 1000 * 5;   // 5 s
    const int n = 2000;
    // warm up
    k_sync<<<1, 64, 0, s>>>(dev, rank, 2, 1, timeout, dev + 64);
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 2; i <= n; ++i) k_sync<<<1, 64, 0, s>>>(dev, rank, 2, unsigned(i), timeout, dev + 64);
    hipStreamSynchronize(s);
    auto t1 = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / (n - 1);
    printf("rank %d: %d back-to-back signal+wait kernels: %.2f us each, err=%u flags=%u,%u\n", rank,
           n - 1, us, host[64], host[0], host[1]);
    // launch-to-completion latency of one sync when the peer is already there
    auto t2 = std::chrono::steady_clock::now();
    for (int i = n + 1; i <= n + 200; ++i) {
        k_sync<<<1, 64, 0, s>>>(dev, rank, 2, unsigned(i), timeout, dev + 64);
        hipStreamSynchronize(s);
    }
    auto t3 = std::chrono::steady_clock::now();
    printf("rank %d: synchronous launch+sync+hostwait: %.2f us each\n", rank,
           std::chrono::duration<double, std::micro>(t3 - t2).count() / 200);
    hipHostUnregister(host);
    return 0;
}

int main() {
    const char *name = "/esgd-probe-flags";
    shm_unlink(name);
    int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, 4096) != 0) { perror("shm"); return 1; }
    unsigned *host = static_cast<unsigned *>(mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
    for (int i = 0; i < 1024; ++i) host[i] = 0;
    pid_t pid = fork();   // before any HIP call
    const int rank = pid == 0 ? 1 : 0;
    int rc = run(rank, host);
    if (pid != 0) {
        int st = 0;
        waitpid(pid, &st, 0);
        shm_unlink(name);
        return rc | (WIFEXITED(st) ? WEXITSTATUS(st) : 1);
    }
    return rc;
}
