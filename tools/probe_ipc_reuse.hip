// probe_ipc_reuse.hip — after an exporter frees an IPC-exported allocation and allocates
// again, (1) do the new handle bytes repeat the old ones, and (2) what does an importer
// that still holds the old mapping get when it opens the new handle?
// Diagnostic only (tools/), not part of the library.  The process forks BEFORE any HIP
// call (no exec); parent = exporter, child = importer, talking over a pipe pair.  The
// importer only reads mappings it holds open.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorName(e_)); _exit(1); } \
    } while (0)

static void hex(const char *tag, const hipIpcMemHandle_t &h) {
    printf("%s", tag);
    const unsigned char *b = reinterpret_cast<const unsigned char *>(&h);
    for (int i = 0; i < 64; ++i) printf("%02x", b[i]);
    printf("\n");
}

static void put(int fd, const void *p, size_t n) { if (write(fd, p, n) != ssize_t(n)) _exit(2); }
static void get(int fd, void *p, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t r = read(fd, static_cast<char *>(p) + got, n - got);
        if (r <= 0) _exit(3);
        got += size_t(r);
    }
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    int to_child[2], to_parent[2];
    if (pipe(to_child) || pipe(to_parent)) return 1;
    const size_t bytes = size_t(16) << 20;
    pid_t pid = fork();
    if (pid == 0) {   // importer
        hipIpcMemHandle_t ha, hb;
        get(to_child[0], &ha, sizeof(ha));
        void *pa = nullptr;
        CK(hipIpcOpenMemHandle(&pa, ha, hipIpcMemLazyEnablePeerAccess));
        unsigned va = 0;
        CK(hipMemcpy(&va, pa, 4, hipMemcpyDeviceToHost));
        printf("importer: A mapped at %p, reads 0x%08x\n", pa, va);
        char ok = 1;
        put(to_parent[1], &ok, 1);
        get(to_child[0], &hb, sizeof(hb));   // exporter freed A, allocated and filled B
        void *pb = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&pb, hb, hipIpcMemLazyEnablePeerAccess);
        printf("importer: open(B) with A still open -> %s, B at %p (%s A)\n", hipGetErrorName(e), pb,
               pb == pa ? "SAME VA as" : "different VA from");
        if (e == hipSuccess) {
            unsigned vb = 0;
            CK(hipMemcpy(&vb, pb, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&va, pa, 4, hipMemcpyDeviceToHost));
            printf("importer: B reads 0x%08x (exporter wrote 0x02020202), A reads 0x%08x\n", vb, va);
        }
        put(to_parent[1], &ok, 1);
        get(to_child[0], &ok, 1);
        CK(hipIpcCloseMemHandle(pa));
        if (e == hipSuccess && pb != pa) CK(hipIpcCloseMemHandle(pb));
        printf("importer: closed\n");
        fflush(stdout);
        put(to_parent[1], &ok, 1);
        _exit(0);
    }
    // exporter
    void *a = nullptr, *b = nullptr, *c = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t ha, hb, hc;
    CK(hipIpcGetMemHandle(&ha, a));
    hex("H(A)  ", ha);
    put(to_child[1], &ha, sizeof(ha));
    char ok;
    get(to_parent[0], &ok, 1);
    CK(hipFree(a));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(b, 2, bytes));
    CK(hipDeviceSynchronize());
    CK(hipIpcGetMemHandle(&hb, b));
    hex("H(B)  ", hb);
    printf("exporter: A at %p, B at %p; handles %s\n", a, b, memcmp(&ha, &hb, 64) ? "DIFFER" : "IDENTICAL");
    put(to_child[1], &hb, sizeof(hb));
    get(to_parent[0], &ok, 1);
    put(to_child[1], &ok, 1);
    get(to_parent[0], &ok, 1);
    CK(hipFree(b));
    CK(hipMalloc(&c, bytes / 2));
    CK(hipIpcGetMemHandle(&hc, c));
    hex("H(C/2)", hc);
    int st = 0;
    waitpid(pid, &st, 0);
    printf("exporter: importer exit %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);
    return 0;
}
