// rm_comm.cpp -- row-sharded frames across GPUs over RCCL (include/rm.h,
// "Multi-GPU").  SURVEY.md 8(b)/8(e): rank r renders the frame rows y with
// (y / band) % nranks == r (rm_render_band_rgba8: RGBA8 packed in the kernel
// epilogue), drops the alpha byte (rm_pack_rgb8: the pass writes alpha 1,
// output_shader.frag:419), one ncclGather brings the 3 B/px bands to rank 0
// over xGMI, and rank 0 de-interleaves them into the RGBA8 frame
// (rm_deinterleave_rgb8).  The gather is the only exchange of the path.
//
// RCCL is opened at run time (dlopen of librccl.so.1): a process that already
// holds one (PyTorch's) shares it, and librm.so itself loads without RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rm.h"
#include "rm_internal.h"
#include "rm_trace.h"

namespace {

// the subset of rccl.h (RCCL 2.2x C API) this file calls
typedef struct ncclComm *ncclComm_t;
typedef struct {
    char internal[128];
} ncclUniqueId;
typedef int ncclResult_t;  // ncclSuccess = 0
constexpr int kNcclUint8 = 1;

struct Rccl {
    void *h = nullptr;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Gather)(const void *, void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl *rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        // an RCCL already in the process (same soname) is reused
        R.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!R.h) R.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!R.h) {
            const char *e = dlerror();
            R.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        auto sym = [](const char *n) { return dlsym(R.h, n); };
        R.GetUniqueId = reinterpret_cast<decltype(R.GetUniqueId)>(sym("ncclGetUniqueId"));
        R.CommInitRank = reinterpret_cast<decltype(R.CommInitRank)>(sym("ncclCommInitRank"));
        R.CommInitAll = reinterpret_cast<decltype(R.CommInitAll)>(sym("ncclCommInitAll"));
        R.CommDestroy = reinterpret_cast<decltype(R.CommDestroy)>(sym("ncclCommDestroy"));
        R.GroupStart = reinterpret_cast<decltype(R.GroupStart)>(sym("ncclGroupStart"));
        R.GroupEnd = reinterpret_cast<decltype(R.GroupEnd)>(sym("ncclGroupEnd"));
        R.Gather = reinterpret_cast<decltype(R.Gather)>(sym("ncclGather"));  // RCCL extension; may be absent
        R.Send = reinterpret_cast<decltype(R.Send)>(sym("ncclSend"));
        R.Recv = reinterpret_cast<decltype(R.Recv)>(sym("ncclRecv"));
        R.GetErrorString = reinterpret_cast<decltype(R.GetErrorString)>(sym("ncclGetErrorString"));
        if (!R.GetUniqueId || !R.CommInitRank || !R.CommInitAll || !R.CommDestroy || !R.GroupStart || !R.GroupEnd ||
            !R.Send || !R.Recv) {
            R.err = "librccl.so.1 lacks a required entry point";
            R.h = nullptr;
        }
    });
    return R.h ? &R : nullptr;
}

}  // namespace

struct rm_comm {
    rm_ctx *ctx = nullptr;
    int nranks = 1, rank = 0;
    ncclComm_t nc = nullptr;
    // buffers of the last frame geometry (reallocated when it grows)
    uint32_t *band = nullptr;    // this rank's packed rows, RGBA8
    uint8_t *wire = nullptr;     // the same rows, RGB8 (rows_per_shard * 3W bytes)
    uint8_t *gathered = nullptr; // root: nranks wires
    size_t band_bytes = 0, wire_bytes = 0, gathered_bytes = 0;
    // render start / render end / gather end / de-interleave end (rm_stats)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
    int rows_mine = 0, rows_per_shard = 0;
    // weighted parts (rm_render_sharded_runs): every rank's rows and the byte
    // offset of its rows in the unpadded gathered buffer
    bool weighted = false;
    std::vector<int> rows_of, base_of;
};

namespace {

rm_status comm_fail(rm_comm *c, rm_status s, const std::string &msg) {
    if (c && c->ctx) rm_internal_set_error(c->ctx, msg);
    return s;
}

rm_status nccl_check(rm_comm *c, ncclResult_t r, const char *what) {
    if (r == 0) return RM_OK;
    Rccl *R = rccl();
    std::string m = std::string(what) + ": " + (R && R->GetErrorString ? R->GetErrorString(r) : "RCCL error");
    return comm_fail(c, RM_ERR_DEVICE, m);
}

template <typename T>
rm_status grow(rm_comm *c, T *&p, size_t &have, size_t need) {
    if (have >= need) return RM_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    have = 0;
    hipError_t e = hipMalloc(&p, need ? need : 1);
    if (e != hipSuccess)
        return comm_fail(c, e == hipErrorOutOfMemory ? RM_ERR_OUT_OF_MEMORY : RM_ERR_DEVICE,
                         std::string("rm_comm buffer: ") + hipGetErrorString(e));
    have = need;
    return RM_OK;
}

rm_status comm_new(rm_comm **out, rm_ctx *ctx, int nranks, int rank) {
    rm_comm *c = new rm_comm();
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    hipError_t e = hipSetDevice(rm_internal_device(ctx));
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e == hipSuccess) e = hipEventCreate(&c->ev2);
    if (e == hipSuccess) e = hipEventCreate(&c->ev3);
    if (e != hipSuccess) {
        rm_comm_destroy(c);
        return RM_ERR_DEVICE;
    }
    *out = c;
    return RM_OK;
}

// How the frame's rows are dealt: round-robin bands of `band` rows, or (runs
// non-null) weighted cyclic parts, rank r owning a run of runs[r] rows in every
// cycle of sum(runs) rows, the runs in rank order.
struct Split {
    int band = 0;
    const int *runs = nullptr;
    int cycle = 0;
    std::vector<int> off;
};
rm_status make_split(rm_comm *c, int band, const int *runs, Split &sp) {
    sp.band = band;
    sp.runs = runs;
    if (!runs) return band > 0 ? RM_OK : RM_ERR_INVALID_ARGUMENT;
    long long cyc = 0;
    sp.off.assign(c->nranks, 0);
    for (int r = 0; r < c->nranks; r++) {
        if (runs[r] < 1) return RM_ERR_INVALID_ARGUMENT;
        sp.off[r] = (int)cyc;
        cyc += runs[r];
        if (cyc > 0x7fffffffLL) return RM_ERR_INVALID_ARGUMENT;
    }
    sp.cycle = (int)cyc;
    return RM_OK;
}

// render + pack this rank's rows (async on the ctx stream)
rm_status enqueue_local(rm_comm *c, int W, int H, const Split &sp) {
    rm_ctx *ctx = c->ctx;
    rm_status st = RM_OK;
    size_t wire_bytes = 0, gathered_bytes = 0;
    c->weighted = sp.runs != nullptr;
    if (!c->weighted) {
        rm_shard_layout L;
        st = rm_sharded_layout(W, H, sp.band, c->nranks, c->rank, &L);
        if (st != RM_OK) return comm_fail(c, st, "rm_render_sharded: bad size/band");
        c->rows_mine = L.rows_mine;
        c->rows_per_shard = L.rows_per_shard;
        wire_bytes = (size_t)L.wire_bytes;
        gathered_bytes = (size_t)L.gathered_bytes;
    } else {
        c->rows_of.assign(c->nranks, 0);
        c->base_of.assign(c->nranks, 0);
        int total = 0;
        for (int r = 0; r < c->nranks; r++) {
            st = rm_cycle_rows(H, sp.cycle, sp.off[r], sp.runs[r], &c->rows_of[r]);
            if (st != RM_OK) return comm_fail(c, st, "rm_render_sharded_runs: bad size/runs");
            c->base_of[r] = total;
            total += c->rows_of[r];
        }
        c->rows_mine = c->rows_of[c->rank];
        c->rows_per_shard = c->rows_mine;
        wire_bytes = (size_t)c->rows_mine * 3 * W;
        gathered_bytes = (size_t)H * 3 * W;  // every row once, rank by rank
    }
    const int n = c->rows_mine;
    if (hipSetDevice(rm_internal_device(ctx)) != hipSuccess) return comm_fail(c, RM_ERR_DEVICE, "hipSetDevice");
    st = grow(c, c->band, c->band_bytes, (size_t)c->rows_per_shard * W * 4);
    if (st == RM_OK) st = grow(c, c->wire, c->wire_bytes, wire_bytes);
    if (st == RM_OK && c->rank == 0 && c->nc) st = grow(c, c->gathered, c->gathered_bytes, gathered_bytes);
    if (st != RM_OK) return st;
    hipStream_t s = rm_internal_stream(ctx);
    if (hipEventRecord(c->ev0, s) != hipSuccess) return comm_fail(c, RM_ERR_DEVICE, "hipEventRecord");
    if (n > 0) {
        st = c->weighted ? rm_render_cycle_rows_rgba8(ctx, W, H, sp.cycle, sp.off[c->rank], sp.runs[c->rank], 0, n,
                                                      c->band, nullptr)
                         : rm_render_band_rgba8(ctx, W, H, sp.band, c->nranks, c->rank, c->band, nullptr);
        if (st != RM_OK) return st;
    }
    if (hipEventRecord(c->ev1, s) != hipSuccess) return comm_fail(c, RM_ERR_DEVICE, "hipEventRecord");
    return rm_pack_rgb8(ctx, (int64_t)n * W, c->band, c->wire);
}

rm_status enqueue_gather_ops(rm_comm *c, int W);

// the gather of every rank's wire into rank 0's gathered buffer, then ev2
rm_status enqueue_gather(rm_comm *c, int W) {
    rm_status st = enqueue_gather_ops(c, W);
    if (st != RM_OK) return st;
    if (hipEventRecord(c->ev2, rm_internal_stream(c->ctx)) != hipSuccess)
        return comm_fail(c, RM_ERR_DEVICE, "hipEventRecord");
    return rm_internal_mark_done(c->ctx);
}

rm_status enqueue_gather_ops(rm_comm *c, int W) {
    if (!c->nc) return RM_OK;  // a one-rank communicator without RCCL: the wire is the gathered buffer
    rm::TraceRange range("rm_gather");
    Rccl *R = rccl();
    hipStream_t s = rm_internal_stream(c->ctx);
    if (c->weighted) {  // unequal parts: grouped point-to-point, unpadded
        const size_t row = (size_t)3 * W;
        rm_status st = nccl_check(c, R->GroupStart(), "ncclGroupStart");
        if (st != RM_OK) return st;
        if (c->rank == 0) {
            for (int r = 1; r < c->nranks && st == RM_OK; r++)
                if (c->rows_of[r] > 0)
                    st = nccl_check(c, R->Recv(c->gathered + (size_t)c->base_of[r] * row, (size_t)c->rows_of[r] * row,
                                               kNcclUint8, r, c->nc, s), "ncclRecv");
        } else if (c->rows_mine > 0) {
            st = nccl_check(c, R->Send(c->wire, (size_t)c->rows_mine * row, kNcclUint8, 0, c->nc, s), "ncclSend");
        }
        rm_status st2 = nccl_check(c, R->GroupEnd(), "ncclGroupEnd");
        if (st != RM_OK) return st;
        if (st2 != RM_OK) return st2;
        if (c->rank == 0 && c->rows_mine > 0 &&
            hipMemcpyAsync(c->gathered, c->wire, (size_t)c->rows_mine * row, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return comm_fail(c, RM_ERR_DEVICE, "gather copy");
        return RM_OK;
    }
    const size_t bytes = (size_t)c->rows_per_shard * 3 * W;
    if (R->Gather)
        return nccl_check(c, R->Gather(c->wire, c->rank == 0 ? c->gathered : nullptr, bytes, kNcclUint8, 0, c->nc, s),
                          "ncclGather");
    // grouped point-to-point form of the gather
    rm_status st = nccl_check(c, R->GroupStart(), "ncclGroupStart");
    if (st != RM_OK) return st;
    if (c->rank == 0) {
        for (int r = 1; r < c->nranks && st == RM_OK; r++)
            st = nccl_check(c, R->Recv(c->gathered + (size_t)r * bytes, bytes, kNcclUint8, r, c->nc, s), "ncclRecv");
    } else {
        st = nccl_check(c, R->Send(c->wire, bytes, kNcclUint8, 0, c->nc, s), "ncclSend");
    }
    rm_status st2 = nccl_check(c, R->GroupEnd(), "ncclGroupEnd");
    if (st != RM_OK) return st;
    if (st2 != RM_OK) return st2;
    if (c->rank == 0 && hipMemcpyAsync(c->gathered, c->wire, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return comm_fail(c, RM_ERR_DEVICE, "gather copy");
    return RM_OK;
}

rm_status finish(rm_comm *c, int W, int H, const Split &sp, uint32_t *frame, rm_stats *stats) {
    rm_status st = RM_OK;
    rm::TraceRange range("rm_deinterleave");
    if (c->rank == 0 && c->weighted) {
        std::vector<int64_t> bytes(c->nranks);
        for (int r = 0; r < c->nranks; r++) bytes[r] = (int64_t)c->base_of[r] * 3 * W;
        st = rm_deinterleave_cycle_rgb8(c->ctx, W, H, sp.cycle, c->nranks, sp.off.data(), sp.runs, bytes.data(),
                                        c->nc ? c->gathered : c->wire, frame);
    } else if (c->rank == 0) {
        st = rm_deinterleave_rgb8(c->ctx, W, H, sp.band, c->nranks, c->rows_per_shard,
                                  c->nc ? c->gathered : c->wire, frame);
    }
    if (st != RM_OK) return st;
    if (c->rank == 0 && hipEventRecord(c->ev3, rm_internal_stream(c->ctx)) != hipSuccess)
        return comm_fail(c, RM_ERR_DEVICE, "hipEventRecord");
    if (!stats) return RM_OK;
    if (hipStreamSynchronize(rm_internal_stream(c->ctx)) != hipSuccess)
        return comm_fail(c, RM_ERR_DEVICE, "hipStreamSynchronize");
    float ms = 0.0f, gms = 0.0f, dms = 0.0f;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    (void)hipEventElapsedTime(&gms, c->ev1, c->ev2);
    if (c->rank == 0) (void)hipEventElapsedTime(&dms, c->ev2, c->ev3);
    std::memset(stats, 0, sizeof(*stats));
    stats->pixels = (uint64_t)W * (uint64_t)c->rows_mine;
    stats->kernel_ms = ms;
    stats->gather_ms = gms;
    stats->deinterleave_ms = dms;
    stats->scene = rm_internal_scene(c->ctx);
    return RM_OK;
}

}  // namespace

extern "C" {

rm_status rm_sharded_layout(int W, int H, int band, int nranks, int rank, rm_shard_layout *out) {
    if (!out || W <= 0 || H <= 0 || band <= 0 || nranks < 1 || rank < 0 || rank >= nranks) return RM_ERR_INVALID_ARGUMENT;
    int n = 0, rps = 0;
    for (int s = 0; s < nranks; s++) {
        int k = 0;
        rm_status st = rm_shard_rows(H, band, nranks, s, &k);
        if (st != RM_OK) return st;
        if (s == rank) n = k;
        rps = k > rps ? k : rps;
    }
    out->rows_mine = n;
    out->rows_per_shard = rps;
    out->wire_bytes = (int64_t)rps * 3 * W;
    out->gathered_bytes = out->wire_bytes * nranks;
    return RM_OK;
}

rm_status rm_comm_get_id(rm_comm_id *id) {
    if (!id) return RM_ERR_INVALID_ARGUMENT;
    Rccl *R = rccl();
    if (!R) return RM_ERR_DEVICE;
    ncclUniqueId u;
    if (R->GetUniqueId(&u) != 0) return RM_ERR_DEVICE;
    static_assert(sizeof(u.internal) == sizeof(id->internal), "rm_comm_id is an ncclUniqueId");
    std::memcpy(id->internal, u.internal, sizeof(u.internal));
    return RM_OK;
}

rm_status rm_comm_init_rank(rm_comm **out, rm_ctx *ctx, int nranks, const rm_comm_id *id, int rank) {
    if (!out || !ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return RM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Rccl *R = rccl();  // a one-rank communicator goes through RCCL too when it loads
    if (nranks > 1 && !R) {
        rm_internal_set_error(ctx, "rm_comm_init_rank: RCCL unavailable");
        return RM_ERR_DEVICE;
    }
    rm_comm *c = nullptr;
    rm_status st = comm_new(&c, ctx, nranks, rank);
    if (st != RM_OK) return st;
    if (R) {
        ncclUniqueId u;
        std::memcpy(u.internal, id->internal, sizeof(u.internal));
        st = nccl_check(c, R->CommInitRank(&c->nc, nranks, u, rank), "ncclCommInitRank");
        if (st != RM_OK) {
            c->nc = nullptr;
            rm_comm_destroy(c);
            return st;
        }
    }
    *out = c;
    return RM_OK;
}

rm_status rm_comm_init_all(rm_comm **comms, rm_ctx *const *ctxs, int n) {
    if (!comms || !ctxs || n < 1) return RM_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n; i++) {
        comms[i] = nullptr;
        if (!ctxs[i]) return RM_ERR_INVALID_ARGUMENT;
    }
    Rccl *R = rccl();
    if (n > 1 && !R) {
        rm_internal_set_error(ctxs[0], "rm_comm_init_all: RCCL unavailable");
        return RM_ERR_DEVICE;
    }
    std::vector<int> devs(n);
    std::vector<ncclComm_t> nc(n, nullptr);
    for (int i = 0; i < n; i++) devs[i] = rm_internal_device(ctxs[i]);
    if (R) {
        ncclResult_t r = R->CommInitAll(nc.data(), n, devs.data());
        if (r != 0) {
            rm_internal_set_error(ctxs[0], std::string("ncclCommInitAll: ") +
                                               (R->GetErrorString ? R->GetErrorString(r) : "RCCL error"));
            return RM_ERR_DEVICE;
        }
    }
    for (int i = 0; i < n; i++) {
        rm_status st = comm_new(&comms[i], ctxs[i], n, i);
        if (st != RM_OK) {
            for (int j = 0; j < n; j++) {
                if (comms[j]) rm_comm_destroy(comms[j]);
                else if (nc[j] && R) R->CommDestroy(nc[j]);
                comms[j] = nullptr;
            }
            return st;
        }
        comms[i]->nc = nc[i];
    }
    return RM_OK;
}

rm_status rm_comm_destroy(rm_comm *c) {
    if (!c) return RM_ERR_INVALID_ARGUMENT;
    if (c->ctx) {
        (void)hipSetDevice(rm_internal_device(c->ctx));
        (void)hipStreamSynchronize(rm_internal_stream(c->ctx));
    }
    if (c->nc) {
        Rccl *R = rccl();
        if (R) R->CommDestroy(c->nc);
    }
    if (c->band) (void)hipFree(c->band);
    if (c->wire) (void)hipFree(c->wire);
    if (c->gathered) (void)hipFree(c->gathered);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->ev3) (void)hipEventDestroy(c->ev3);
    delete c;
    return RM_OK;
}

rm_status rm_comm_info(const rm_comm *comm, int *nranks, int *rank, int *uses_rccl) {
    if (!comm) return RM_ERR_INVALID_ARGUMENT;
    if (nranks) *nranks = comm->nranks;
    if (rank) *rank = comm->rank;
    if (uses_rccl) *uses_rccl = comm->nc != nullptr;
    return RM_OK;
}

}  // extern "C"

namespace {

rm_status render_sharded(rm_comm *comm, int W, int H, int band, const int *runs, uint32_t *frame, rm_stats *stats) {
    if (!comm) return RM_ERR_INVALID_ARGUMENT;
    Split sp;
    if (W <= 0 || H <= 0 || make_split(comm, band, runs, sp) != RM_OK)
        return comm_fail(comm, RM_ERR_INVALID_ARGUMENT, "rm_render_sharded: bad size/band/runs");
    if (comm->rank == 0 && !frame) return comm_fail(comm, RM_ERR_INVALID_ARGUMENT, "rm_render_sharded: null frame on rank 0");
    rm_status st = enqueue_local(comm, W, H, sp);
    if (st == RM_OK) st = enqueue_gather(comm, W);
    if (st == RM_OK) st = finish(comm, W, H, sp, frame, stats);
    return st;
}

rm_status render_sharded_all(rm_comm *const *comms, int n, int W, int H, int band, const int *runs, uint32_t *frame,
                             rm_stats *stats) {
    if (!comms || n < 1 || !frame) return RM_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n; i++)
        if (!comms[i] || comms[i]->nranks != n || comms[i]->rank != i) return RM_ERR_INVALID_ARGUMENT;
    Split sp;
    if (W <= 0 || H <= 0 || make_split(comms[0], band, runs, sp) != RM_OK)
        return comm_fail(comms[0], RM_ERR_INVALID_ARGUMENT, "rm_render_sharded_all: bad size/band/runs");
    for (int i = 0; i < n; i++) {  // every device renders its rows concurrently
        rm_status st = enqueue_local(comms[i], W, H, sp);
        if (st != RM_OK) return st;
    }
    if (n == 1) {
        rm_status st = enqueue_gather(comms[0], W);
        if (st != RM_OK) return st;
    } else {
        // one group: the n gathers (one per device) complete as one collective
        Rccl *R = rccl();
        rm_status st = nccl_check(comms[0], R->GroupStart(), "ncclGroupStart");
        for (int i = 0; i < n && st == RM_OK; i++) {
            (void)hipSetDevice(rm_internal_device(comms[i]->ctx));
            st = enqueue_gather_ops(comms[i], W);
        }
        rm_status st2 = nccl_check(comms[0], R->GroupEnd(), "ncclGroupEnd");
        if (st != RM_OK) return st;
        if (st2 != RM_OK) return st2;
        // the grouped gathers reach the streams at ncclGroupEnd: their end events after it
        for (int i = 0; i < n; i++) {
            (void)hipSetDevice(rm_internal_device(comms[i]->ctx));
            if (hipEventRecord(comms[i]->ev2, rm_internal_stream(comms[i]->ctx)) != hipSuccess)
                return comm_fail(comms[i], RM_ERR_DEVICE, "hipEventRecord");
            st = rm_internal_mark_done(comms[i]->ctx);
            if (st != RM_OK) return st;
        }
    }
    (void)hipSetDevice(rm_internal_device(comms[0]->ctx));
    for (int i = 0; i < n; i++) {
        rm_status st = finish(comms[i], W, H, sp, i == 0 ? frame : nullptr, stats ? stats + i : nullptr);
        if (st != RM_OK) return st;
    }
    return RM_OK;
}

}  // namespace

extern "C" {

rm_status rm_render_sharded(rm_comm *comm, int W, int H, int band, uint32_t *frame, rm_stats *stats) {
    return render_sharded(comm, W, H, band, nullptr, frame, stats);
}

rm_status rm_render_sharded_all(rm_comm *const *comms, int n, int W, int H, int band, uint32_t *frame,
                                rm_stats *stats) {
    return render_sharded_all(comms, n, W, H, band, nullptr, frame, stats);
}

rm_status rm_render_sharded_runs(rm_comm *comm, int W, int H, const int *runs, uint32_t *frame, rm_stats *stats) {
    if (!comm) return RM_ERR_INVALID_ARGUMENT;
    if (!runs) return comm_fail(comm, RM_ERR_INVALID_ARGUMENT, "rm_render_sharded_runs: null runs");
    return render_sharded(comm, W, H, 0, runs, frame, stats);
}

rm_status rm_render_sharded_runs_all(rm_comm *const *comms, int n, int W, int H, const int *runs, uint32_t *frame,
                                     rm_stats *stats) {
    if (!runs) return RM_ERR_INVALID_ARGUMENT;
    return render_sharded_all(comms, n, W, H, 0, runs, frame, stats);
}

}  // extern "C"
