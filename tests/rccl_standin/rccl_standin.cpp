// rccl_standin.cpp -- TEST INFRASTRUCTURE ONLY: a stand-in for librccl.so.1
// that lets librm.so's N > 1 multi-GPU path (rm_comm.cpp: rm_comm_init_all +
// rm_render_sharded_all, rm_comm_init_rank + rm_render_sharded) run on a box
// with ONE GPU, where real RCCL refuses two ranks on the same device.
//
// It exports the RCCL C API subset librm.so resolves with dlsym
// (ncclGetUniqueId, ncclCommInitRank, ncclCommInitAll, ncclCommDestroy,
// ncclGroupStart/End, ncclGather, ncclSend, ncclRecv, ncclGetErrorString) and
// moves the bytes itself:
//   * ranks of one process (ncclCommInitAll): at ncclGroupEnd every matched
//     gather / send-recv becomes hipMemcpyAsync on the receiver's stream after
//     an event of the sender's stream, and the sender's stream then waits for
//     the copies (the stream semantics of a collective);
//   * ranks in separate processes (ncclCommInitRank): a POSIX shared-memory
//     segment named by the unique id, one slot per rank; a sender waits for
//     its stream and copies its buffer into its slot, the receiver copies the
//     slot into its buffer (blocking calls; sequence counters per rank).
// Built twice (tests/rccl_standin/Makefile): with ncclGather, and without it
// (-DSTANDIN_NO_GATHER) so that librm.so takes its grouped send/recv form.
// Only tests put it on LD_LIBRARY_PATH of a driver process; the product never
// loads it.  rccl_standin_stats counts the operations it carried out.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

typedef int ncclResult_t;
enum {
    ncclSuccess = 0,
    ncclUnhandledCudaError = 1,
    ncclSystemError = 2,
    ncclInternalError = 3,
    ncclInvalidArgument = 4,
    ncclInvalidUsage = 5
};
typedef struct {
    char internal[128];
} ncclUniqueId;

namespace {

constexpr int kMaxRanks = 64;
constexpr uint32_t kMagic = 0x524d5349u;  // "RMSI"

struct ShmHdr {
    uint32_t magic;
    int nranks;
    uint64_t slot_bytes;
    std::atomic<int> joined;
    std::atomic<int> left;
    std::atomic<uint64_t> posted[kMaxRanks];    // messages rank r has placed in its slot
    std::atomic<uint64_t> consumed[kMaxRanks];  // messages of rank r its receiver has taken
    int dst[kMaxRanks];                         // receiver of rank r's posted message
    uint64_t bytes[kMaxRanks];
};

struct World;

}  // namespace

struct ncclComm {
    int nranks = 1, rank = 0, dev = 0;
    World *world = nullptr;  // ranks of this process (ncclCommInitAll)
    ShmHdr *shm = nullptr;   // ranks in separate processes (ncclCommInitRank)
    size_t shm_size = 0;
    std::string shm_name;
    uint64_t recv_seq[kMaxRanks] = {};  // messages taken from each source
};
typedef ncclComm *ncclComm_t;

extern "C" {
// gathers, sends, recvs, grouped flushes carried out (tests read it with dlsym)
unsigned long long rccl_standin_stats[4] = {0, 0, 0, 0};
}

namespace {

struct World {
    int n = 0;
    std::vector<ncclComm *> comms;
};

enum Kind { GATHER, SEND, RECV };
struct Op {
    Kind kind;
    ncclComm *c;
    const void *sbuf;
    void *rbuf;
    size_t bytes;
    int peer;  // root (gather) or the other rank (send / recv)
    hipStream_t s;
};

thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

double timeout_s() {
    const char *e = std::getenv("RCCL_STANDIN_TIMEOUT");
    return e ? std::atof(e) : 120.0;
}

template <typename F>
bool wait_until(F ready) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!ready()) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s()) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    return true;
}

// dst (on dst's stream) <- src (on src's stream): the copy waits for src's
// stream; src's stream then waits for the copy
ncclResult_t stream_copy(void *dst, int ddev, hipStream_t ds, const void *src, int sdev, hipStream_t ss, size_t n) {
    hipEvent_t ready = nullptr, done = nullptr;
    if (hipSetDevice(sdev) != hipSuccess || hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(ready, ss) != hipSuccess)
        return ncclUnhandledCudaError;
    hipError_t e = hipSetDevice(ddev);
    if (e == hipSuccess) e = hipStreamWaitEvent(ds, ready, 0);
    if (e == hipSuccess && n) e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, ds);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(done, ds);
    if (e == hipSuccess) e = hipSetDevice(sdev);
    if (e == hipSuccess) e = hipStreamWaitEvent(ss, done, 0);
    (void)hipEventDestroy(ready);
    if (done) (void)hipEventDestroy(done);
    return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

// ---- in-process ranks: matched at the end of the group
ncclResult_t run_world(std::vector<Op> &ops) {
    for (Op &o : ops) {
        if (o.kind == GATHER && o.c->rank == o.peer) {  // the root's gather pulls every rank's buffer
            const World *w = o.c->world;
            for (int r = 0; r < w->n; r++) {
                const Op *src = nullptr;
                for (const Op &p : ops)
                    if (p.kind == GATHER && p.c->world == w && p.c->rank == r && p.peer == o.peer) src = &p;
                if (!src || src->bytes != o.bytes) return ncclInvalidUsage;  // a rank did not join the gather
                ncclResult_t res = stream_copy(static_cast<char *>(o.rbuf) + (size_t)r * o.bytes, o.c->dev, o.s,
                                               src->sbuf, src->c->dev, src->s, o.bytes);
                if (res != ncclSuccess) return res;
            }
            rccl_standin_stats[0]++;
        } else if (o.kind == RECV) {
            const Op *src = nullptr;
            for (const Op &p : ops)
                if (p.kind == SEND && p.c->world == o.c->world && p.c->rank == o.peer && p.peer == o.c->rank) src = &p;
            if (!src || src->bytes != o.bytes) return ncclInvalidUsage;
            ncclResult_t res = stream_copy(o.rbuf, o.c->dev, o.s, src->sbuf, src->c->dev, src->s, o.bytes);
            if (res != ncclSuccess) return res;
            rccl_standin_stats[1]++;
            rccl_standin_stats[2]++;
        }
    }
    return ncclSuccess;
}

// ---- ranks in separate processes: slots of the shared segment
char *slot(ncclComm *c, int r) {
    return reinterpret_cast<char *>(c->shm) + sizeof(ShmHdr) + (size_t)r * c->shm->slot_bytes;
}

ncclResult_t shm_send(ncclComm *c, const void *buf, size_t n, int dst, hipStream_t s) {
    ShmHdr *h = c->shm;
    if (n > h->slot_bytes) return ncclInvalidArgument;
    const int r = c->rank;
    const uint64_t k = h->posted[r].load() + 1;
    if (!wait_until([&] { return h->consumed[r].load() == k - 1; })) return ncclSystemError;  // slot free
    if (hipSetDevice(c->dev) != hipSuccess || hipStreamSynchronize(s) != hipSuccess ||
        (n && hipMemcpy(slot(c, r), buf, n, hipMemcpyDeviceToHost) != hipSuccess))
        return ncclUnhandledCudaError;
    h->dst[r] = dst;
    h->bytes[r] = n;
    h->posted[r].store(k);
    return ncclSuccess;
}

ncclResult_t shm_recv(ncclComm *c, void *buf, size_t n, int src, hipStream_t s) {
    ShmHdr *h = c->shm;
    const uint64_t k = c->recv_seq[src] + 1;
    if (!wait_until([&] { return h->posted[src].load() >= k; })) return ncclSystemError;
    if (h->dst[src] != c->rank || h->bytes[src] != n) return ncclInvalidUsage;
    if (hipSetDevice(c->dev) != hipSuccess || hipStreamSynchronize(s) != hipSuccess ||
        (n && hipMemcpy(buf, slot(c, src), n, hipMemcpyHostToDevice) != hipSuccess))
        return ncclUnhandledCudaError;
    c->recv_seq[src] = k;
    h->consumed[src].store(k);
    return ncclSuccess;
}

ncclResult_t run_shm(std::vector<Op> &ops) {
    // sends first (they never wait for this process's receives), then receives
    for (int pass = 0; pass < 2; pass++)
        for (Op &o : ops) {
            ncclResult_t r = ncclSuccess;
            if (o.kind == GATHER) {
                if (pass == 0 && o.c->rank != o.peer) {
                    r = shm_send(o.c, o.sbuf, o.bytes, o.peer, o.s);
                } else if (pass == 1 && o.c->rank == o.peer) {
                    r = stream_copy(static_cast<char *>(o.rbuf) + (size_t)o.c->rank * o.bytes, o.c->dev, o.s,
                                    o.sbuf, o.c->dev, o.s, o.bytes);
                    for (int q = 0; q < o.c->nranks && r == ncclSuccess; q++)
                        if (q != o.c->rank) r = shm_recv(o.c, static_cast<char *>(o.rbuf) + (size_t)q * o.bytes, o.bytes, q, o.s);
                    if (r == ncclSuccess) rccl_standin_stats[0]++;
                }
            } else if (o.kind == SEND && pass == 0) {
                r = shm_send(o.c, o.sbuf, o.bytes, o.peer, o.s);
                if (r == ncclSuccess) rccl_standin_stats[1]++;
            } else if (o.kind == RECV && pass == 1) {
                r = shm_recv(o.c, o.rbuf, o.bytes, o.peer, o.s);
                if (r == ncclSuccess) rccl_standin_stats[2]++;
            }
            if (r != ncclSuccess) return r;
        }
    return ncclSuccess;
}

ncclResult_t flush() {
    std::vector<Op> ops;
    ops.swap(g_ops);
    if (ops.empty()) return ncclSuccess;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::vector<Op> local, shm;
    for (Op &o : ops) (o.c->world ? local : shm).push_back(o);
    ncclResult_t r = run_world(local);
    if (r == ncclSuccess) r = run_shm(shm);
    (void)hipSetDevice(dev);
    rccl_standin_stats[3]++;
    return r;
}

ncclResult_t enqueue(const Op &o) {
    if (!o.c || o.peer < 0 || o.peer >= o.c->nranks) return ncclInvalidArgument;
    g_ops.push_back(o);
    if (g_depth > 0) return ncclSuccess;
    // outside a group an in-process collective of several ranks cannot complete
    // (the other ranks' calls come later from this same thread)
    if (o.c->world && o.c->nranks > 1) {
        g_ops.clear();
        return ncclInvalidUsage;
    }
    return flush();
}

}  // namespace

extern "C" {

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "no error (rccl stand-in)";
    case ncclUnhandledCudaError: return "HIP call failed (rccl stand-in)";
    case ncclSystemError: return "timed out waiting for a peer (rccl stand-in)";
    case ncclInvalidArgument: return "invalid argument (rccl stand-in)";
    case ncclInvalidUsage: return "invalid usage (rccl stand-in)";
    default: return "internal error (rccl stand-in)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    static std::atomic<int> counter{0};
    std::memset(id->internal, 0, sizeof(id->internal));
    const long long t = (long long)std::chrono::steady_clock::now().time_since_epoch().count();
    std::snprintf(id->internal, sizeof(id->internal), "/rmsi_%d_%d_%llx", (int)getpid(), counter++, t);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks || id.internal[0] != '/')
        return ncclInvalidArgument;
    ncclComm *c = new ncclComm();
    c->nranks = nranks;
    c->rank = rank;
    (void)hipGetDevice(&c->dev);
    const char *e = std::getenv("RCCL_STANDIN_SLOT_BYTES");
    const uint64_t slot_bytes = e ? std::strtoull(e, nullptr, 10) : (64ull << 20);
    c->shm_name.assign(id.internal, strnlen(id.internal, sizeof(id.internal)));
    c->shm_size = sizeof(ShmHdr) + (size_t)nranks * slot_bytes;
    const int fd = shm_open(c->shm_name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)c->shm_size) != 0) {
        if (fd >= 0) close(fd);
        delete c;
        return ncclSystemError;
    }
    void *p = mmap(nullptr, c->shm_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        delete c;
        return ncclSystemError;
    }
    c->shm = static_cast<ShmHdr *>(p);
    // the segment starts zeroed (ftruncate): rank 0 stamps it, the others wait
    if (rank == 0) {
        c->shm->nranks = nranks;
        c->shm->slot_bytes = slot_bytes;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        reinterpret_cast<std::atomic<uint32_t> *>(&c->shm->magic)->store(kMagic);
    }
    ShmHdr *h = c->shm;
    bool ok = wait_until([&] { return reinterpret_cast<std::atomic<uint32_t> *>(&h->magic)->load() == kMagic; }) &&
              h->nranks == nranks && h->slot_bytes == slot_bytes;
    if (ok) {
        h->joined.fetch_add(1);
        ok = wait_until([&] { return h->joined.load() >= nranks; });  // init is collective
    }
    if (!ok) {
        munmap(p, c->shm_size);
        delete c;
        return ncclSystemError;
    }
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comms, int n, const int *devs) {
    if (!comms || n < 1 || n > kMaxRanks) return ncclInvalidArgument;
    World *w = new World();
    w->n = n;
    for (int i = 0; i < n; i++) {
        ncclComm *c = new ncclComm();
        c->nranks = n;
        c->rank = i;
        c->dev = devs ? devs[i] : i;
        c->world = w;
        w->comms.push_back(c);
        comms[i] = c;
    }
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    if (c->shm) {
        const bool last = c->shm->left.fetch_add(1) + 1 == c->nranks;
        munmap(c->shm, c->shm_size);
        if (last) shm_unlink(c->shm_name.c_str());
    }
    if (c->world) {
        World *w = c->world;
        for (ncclComm *&p : w->comms)
            if (p == c) p = nullptr;
        bool empty = true;
        for (ncclComm *p : w->comms) empty &= p == nullptr;
        if (empty) delete w;
    }
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    g_depth++;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    return --g_depth == 0 ? flush() : ncclSuccess;
}

#ifndef STANDIN_NO_GATHER
// RCCL's gather extension: root receives nranks * count bytes (uint8 only here)
ncclResult_t ncclGather(const void *sbuf, void *rbuf, size_t count, int dtype, int root, ncclComm_t c, hipStream_t s) {
    if (dtype != 1 && dtype != 0) return ncclInvalidArgument;  // ncclInt8 / ncclUint8
    if (c && c->rank == root && !rbuf) return ncclInvalidArgument;
    return enqueue(Op{GATHER, c, sbuf, rbuf, count, root, s});
}
#endif

ncclResult_t ncclSend(const void *buf, size_t count, int dtype, int peer, ncclComm_t c, hipStream_t s) {
    if (dtype != 1 && dtype != 0) return ncclInvalidArgument;
    return enqueue(Op{SEND, c, buf, nullptr, count, peer, s});
}

ncclResult_t ncclRecv(void *buf, size_t count, int dtype, int peer, ncclComm_t c, hipStream_t s) {
    if (dtype != 1 && dtype != 0) return ncclInvalidArgument;
    return enqueue(Op{RECV, c, nullptr, buf, count, peer, s});
}

}  // extern "C"
