// arena.cpp — device memory for buckets that peers map over IPC.
//
// The data plane shares buckets between the node's processes through hipIpc handles.
// Measured on MI355X ("IPC arena"): once a bucket that had been exported
// and mapped by peers is freed and its pages are handed to a new allocation that is
// exported again, peers reading the new bucket through their fresh mappings (and the
// owner's own results) come out wrong -- 8 ranks, a 16 MiB bucket freed, then a 256 MiB
// one: every round mismatched; with the first bucket kept alive, or allocated after the
// second, every round was bit-exact.  Round 1 saw the same family as illegal memory
// accesses after re-opening handle bytes and after freeing exported memory.
//
// So exported memory is never freed while the process runs: esgd_malloc / esgd_free and
// every bucket the library owns come from this arena.  A freed block goes back to a free
// list of its size class and is handed out again in this process; its chunk (one
// hipMalloc) is exported once, each peer maps it once and keeps the mapping until
// finalize.  Foreign device memory (torch tensors, plain hipMalloc) is never exported:
// schedules over it reduce through an arena bucket (the shadow path, dataplane.cpp).
//
// Size classes: powers of two from 4 KiB to 1 MiB carved out of 2 MiB slabs; larger
// blocks are chunks of their own, rounded up to 2 MiB, reused for requests within 25 %
// of their size.  Chunks that were never exported go back to the driver when an
// allocation fails and at finalize (arena_trim).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "esgd_internal.h"

namespace esgd {

namespace {

constexpr size_t kSlab = size_t(2) << 20;
constexpr size_t kMinBlock = 4096;

struct Chunk {
    char *base = nullptr;
    size_t bytes = 0;
    int device = -1;
    bool exported = false;
    uint8_t handle[64] = {};
    int live = 0;          // blocks handed out and not freed
};

struct Block {
    Chunk *chunk;
    size_t cls;            // bytes of the block
};

std::mutex g_mu;
std::vector<Chunk *> g_chunks;
std::map<uintptr_t, Block> g_live;                        // block start -> block
std::map<std::pair<int, size_t>, std::vector<char *>> g_small;   // (device, class) -> free blocks
std::multimap<std::pair<int, size_t>, char *> g_large;   // (device, bytes) -> free chunks
std::map<uintptr_t, Chunk *> g_by_base;                   // chunk base -> chunk

size_t small_class(size_t bytes) {
    size_t c = kMinBlock;
    while (c < bytes) c <<= 1;
    return c;
}

int new_chunk(size_t bytes, int dev, Chunk **out) {
    char *p = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), bytes);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        // give never-exported free chunks back and retry once
        for (auto it = g_large.begin(); it != g_large.end();) {
            auto c = g_by_base.find(reinterpret_cast<uintptr_t>(it->second));
            if (c != g_by_base.end() && !c->second->exported && c->second->device == dev) {
                (void)hipFree(c->second->base);
                g_chunks.erase(std::remove(g_chunks.begin(), g_chunks.end(), c->second), g_chunks.end());
                delete c->second;
                g_by_base.erase(c);
                it = g_large.erase(it);
            } else {
                ++it;
            }
        }
        e = hipMalloc(reinterpret_cast<void **>(&p), bytes);
    }
    if (e != hipSuccess) return hip_fail(e, "hipMalloc (bucket arena)", __FILE__, __LINE__);
    auto *c = new Chunk();
    c->base = p;
    c->bytes = bytes;
    c->device = dev;
    g_chunks.push_back(c);
    g_by_base[reinterpret_cast<uintptr_t>(p)] = c;
    *out = c;
    return ESGD_SUCCESS;
}

}  // namespace

int arena_alloc(size_t bytes, void **out) {
    ESGD_ARG(out, "arena: null output");
    if (int rc = require_device()) return rc;
    int dev = 0;
    ESGD_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_mu);
    bytes = std::max<size_t>(bytes, 1);
    if (bytes <= kSlab / 2) {
        const size_t cls = small_class(bytes);
        auto &fl = g_small[{dev, cls}];
        if (fl.empty()) {
            Chunk *c = nullptr;
            if (int rc = new_chunk(kSlab, dev, &c)) return rc;
            for (size_t o = kSlab; o >= cls; o -= cls) fl.push_back(c->base + o - cls);
        }
        char *p = fl.back();
        fl.pop_back();
        auto base = g_by_base.upper_bound(reinterpret_cast<uintptr_t>(p));
        --base;
        Chunk *c = base->second;
        ++c->live;
        g_live[reinterpret_cast<uintptr_t>(p)] = {c, cls};
        *out = p;
        return ESGD_SUCCESS;
    }
    const size_t need = (bytes + kSlab - 1) / kSlab * kSlab;
    auto it = g_large.lower_bound({dev, need});
    if (it != g_large.end() && it->first.first == dev && it->first.second <= need + need / 4) {
        char *p = it->second;
        g_large.erase(it);
        Chunk *c = g_by_base[reinterpret_cast<uintptr_t>(p)];
        ++c->live;
        g_live[reinterpret_cast<uintptr_t>(p)] = {c, c->bytes};
        *out = p;
        return ESGD_SUCCESS;
    }
    Chunk *c = nullptr;
    if (int rc = new_chunk(need, dev, &c)) return rc;
    ++c->live;
    g_live[reinterpret_cast<uintptr_t>(c->base)] = {c, need};
    *out = c->base;
    return ESGD_SUCCESS;
}

// true if p was handed out by the arena (it is back on a free list now)
bool arena_free(void *p) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.find(reinterpret_cast<uintptr_t>(p));
    if (it == g_live.end()) return false;
    Block b = it->second;
    g_live.erase(it);
    --b.chunk->live;
    if (b.cls <= kSlab / 2) g_small[{b.chunk->device, b.cls}].push_back(static_cast<char *>(p));
    else g_large.insert({{b.chunk->device, b.chunk->bytes}, static_cast<char *>(p)});
    return true;
}

// The arena chunk holding [p, p + bytes) of a live block: its base, the offset of p and
// its IPC handle (created on first use; the chunk is marked exported and is never given
// back to the driver while the process runs).  ESGD_INVALID_ARG if p is not arena memory.
int arena_export(const void *p, size_t bytes, void **base, uint64_t *off, uint8_t handle[64]) {
    std::lock_guard<std::mutex> lk(g_mu);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = g_live.upper_bound(a);
    if (it == g_live.begin()) return ESGD_INVALID_ARG;
    --it;
    const Block &b = it->second;
    if (a + bytes > it->first + b.cls) return ESGD_INVALID_ARG;
    Chunk *c = b.chunk;
    if (!c->exported) {
        hipIpcMemHandle_t h;
        if (hipError_t e = hipIpcGetMemHandle(&h, c->base)) {
            const char *m = getenv("HSA_ENABLE_IPC_MODE_LEGACY");
            int rc = hip_fail(e, "hipIpcGetMemHandle", __FILE__, __LINE__);
            if (!m || std::strcmp(m, "0") != 0) {
                std::string msg = esgd_last_error();
                set_error("%s -- this node's driver exports only dmabuf handles: set "
                          "HSA_ENABLE_IPC_MODE_LEGACY=0 in every rank's environment", msg.c_str());
            }
            return rc;
        }
        std::memcpy(c->handle, &h, 64);
        c->exported = true;
    }
    *base = c->base;
    *off = uint64_t(a - reinterpret_cast<uintptr_t>(c->base));
    std::memcpy(handle, c->handle, 64);
    return ESGD_SUCCESS;
}

// Finalize: chunks that were never exported and hold no live block go back to the
// driver.  Exported chunks stay until the process exits: a peer may still hold a mapping
// (and freeing exported memory is what this arena exists to avoid).
void arena_trim() {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto it = g_chunks.begin(); it != g_chunks.end();) {
        Chunk *c = *it;
        if (c->exported || c->live) { ++it; continue; }
        for (auto fl = g_small.begin(); fl != g_small.end(); ++fl) {
            auto &v = fl->second;
            v.erase(std::remove_if(v.begin(), v.end(), [&](char *p) { return p >= c->base && p < c->base + c->bytes; }),
                    v.end());
        }
        for (auto fl = g_large.begin(); fl != g_large.end();) {
            if (fl->second == c->base) fl = g_large.erase(fl);
            else ++fl;
        }
        g_by_base.erase(reinterpret_cast<uintptr_t>(c->base));
        (void)hipFree(c->base);
        delete c;
        it = g_chunks.erase(it);
    }
}

}  // namespace esgd
