// shard_driver.cpp -- TEST INFRASTRUCTURE ONLY: drives librm.so's multi-GPU
// C ABI (include/rm.h "Multi-GPU") without Python or torch, so that a test can
// put the RCCL stand-in (rccl_standin.cpp) on LD_LIBRARY_PATH, or run it over
// the real RCCL on a multi-GPU node.
//
//   shard_driver all   N W H BAND SCENE   one process, N contexts (rm_comm_init_all
//                                          + rm_render_sharded_all)
//   shard_driver ranks N W H BAND SCENE   N processes, one context each
//                                          (rm_comm_get_id, rm_comm_init_rank,
//                                          rm_render_sharded)
// Contexts use device i % device_count (RM_DRIVER_ONE_DEVICE=1: all on device 0).
// Each renders two frames at two poses; rank 0's gathered RGBA8 frame must equal
// rm_render_rgba8 of a plain context at the same pose, byte for byte.  Prints
// one JSON line; exit 0 when every frame is equal.
//
// The ranks mode forks its N workers before anything touches the GPU (the
// parent never does); rank 0's worker creates the unique id and hands it to the
// others through shared memory.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rm.h"

namespace {

struct Pose {
    float pos[3], mouse[2], time;
};
// raymarching_amd/poses.py P3 and P4
const Pose kPoses[2] = {
    {{0.49591487646102905f, 5.587482452392578f, 6.250702381134033f}, {-0.6590452194213867f, 0.1154678612947464f},
     177.62171936035156f},
    {{0.1990164816379547f, 5.769715785980225f, 2.443920135498047f}, {-0.30864861607551575f, -0.47235697507858276f},
     57.79888153076172f}};

int g_W, g_H, g_band;
std::vector<int> g_runs;  // BAND given as "r0,r1,...": weighted parts (rm_render_sharded_runs*)
std::string g_scene;

bool setup(rm_ctx *c, const Pose &p) {
    rm_params prm;
    return rm_get_params(c, &prm) == RM_OK && (prm.max_steps = 128, prm.schedule = 1, rm_set_params(c, &prm) == RM_OK) &&
           rm_set_uniform3f(c, "u_pos", p.pos[0], p.pos[1], p.pos[2]) == RM_OK &&
           rm_set_uniform2f(c, "u_mouse", p.mouse[0], p.mouse[1]) == RM_OK &&
           rm_set_uniform1f(c, "u_time", p.time) == RM_OK;
}

int device_for(int i) {
    if (const char *e = std::getenv("RM_DRIVER_ONE_DEVICE"); e && std::atoi(e)) return 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 0;
    return i % n;
}

// the reference frame: a plain context on the root's device
bool reference(int dev, const Pose &p, std::vector<uint32_t> &out) {
    rm_ctx *c = nullptr;
    if (rm_create(&c, dev) != RM_OK) return false;
    uint32_t *d = nullptr;
    out.resize((size_t)g_W * g_H);
    bool ok = rm_load_scene(c, g_scene.c_str()) == RM_OK && setup(c, p) &&
              hipMalloc(&d, out.size() * 4) == hipSuccess && rm_render_rgba8(c, g_W, g_H, d, nullptr) == RM_OK &&
              rm_synchronize(c) == RM_OK && hipMemcpy(out.data(), d, out.size() * 4, hipMemcpyDeviceToHost) == hipSuccess;
    if (d) (void)hipFree(d);
    rm_destroy(c);
    return ok;
}

std::string standin_stats() {
    auto *s = static_cast<unsigned long long *>(dlsym(RTLD_DEFAULT, "rccl_standin_stats"));
    if (!s) return "null";
    char b[128];
    std::snprintf(b, sizeof(b), "[%llu, %llu, %llu, %llu]", s[0], s[1], s[2], s[3]);
    return b;
}

int run_all(int n) {
    std::vector<rm_ctx *> ctx(n, nullptr);
    std::vector<rm_comm *> comm(n, nullptr);
    for (int i = 0; i < n; i++)
        if (rm_create(&ctx[i], device_for(i)) != RM_OK || rm_load_scene(ctx[i], g_scene.c_str()) != RM_OK) {
            std::fprintf(stderr, "context %d: %s\n", i, ctx[i] ? rm_last_error(ctx[i]) : "rm_create");
            return 1;
        }
    if (rm_comm_init_all(comm.data(), ctx.data(), n) != RM_OK) {
        std::fprintf(stderr, "rm_comm_init_all: %s\n", rm_last_error(ctx[0]));
        return 1;
    }
    int uses = 0;
    rm_comm_info(comm[0], nullptr, nullptr, &uses);
    const int root_dev = device_for(0);
    (void)hipSetDevice(root_dev);
    uint32_t *frame = nullptr;
    if (hipMalloc(&frame, (size_t)g_W * g_H * 4) != hipSuccess) return 1;
    bool equal = true;
    int frames = 0;
    std::vector<rm_stats> st(n);
    for (int f = 0; f < 2; f++) {
        for (int i = 0; i < n; i++)
            if (!setup(ctx[i], kPoses[f])) return 1;
        const rm_status rs = g_runs.empty() ? rm_render_sharded_all(comm.data(), n, g_W, g_H, g_band, frame, st.data())
                                            : rm_render_sharded_runs_all(comm.data(), n, g_W, g_H, g_runs.data(), frame,
                                                                         st.data());
        if (rs != RM_OK) {
            std::fprintf(stderr, "rm_render_sharded_all: %s\n", rm_last_error(ctx[0]));
            return 1;
        }
        std::vector<uint32_t> got((size_t)g_W * g_H), ref;
        (void)hipSetDevice(root_dev);
        if (rm_synchronize(ctx[0]) != RM_OK ||
            hipMemcpy(got.data(), frame, got.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
            !reference(root_dev, kPoses[f], ref))
            return 1;
        equal &= got == ref;
        frames++;
    }
    std::printf("{\"mode\": \"all\", \"n\": %d, \"W\": %d, \"H\": %d, \"band\": %d, \"frames\": %d, \"equal\": %s, "
                "\"uses_rccl\": %d, \"standin_stats\": %s, \"root_ms\": [%g, %g, %g], \"last_rank_ms\": [%g, %g, %g]}\n",
                n, g_W, g_H, g_band, frames, equal ? "true" : "false", uses, standin_stats().c_str(), st[0].kernel_ms,
                st[0].gather_ms, st[0].deinterleave_ms, st[n - 1].kernel_ms, st[n - 1].gather_ms,
                st[n - 1].deinterleave_ms);
    for (rm_comm *c : comm) rm_comm_destroy(c);
    (void)hipFree(frame);
    for (rm_ctx *c : ctx) rm_destroy(c);
    return equal ? 0 : 3;
}

struct Shared {  // MAP_SHARED | MAP_ANONYMOUS, created before the fork
    std::atomic<int> id_ready;
    rm_comm_id id;
    std::atomic<int> equal;
    std::atomic<int> frames;
    std::atomic<int> uses_rccl;
    char stats[128];
    float root_ms[3];  // rank 0's rm_stats of the last frame: kernel, gather, de-interleave
};

int rank_worker(Shared *sh, int n, int rank) {
    if (rank == 0) {
        if (rm_comm_get_id(&sh->id) != RM_OK) {
            std::fprintf(stderr, "rm_comm_get_id failed\n");
            sh->id_ready.store(-1);
            return 1;
        }
        sh->id_ready.store(1);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while (sh->id_ready.load() == 0) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return 1;
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (sh->id_ready.load() < 0) return 1;
    }
    const int dev = device_for(rank);
    rm_ctx *ctx = nullptr;
    rm_comm *comm = nullptr;
    if (rm_create(&ctx, dev) != RM_OK || rm_load_scene(ctx, g_scene.c_str()) != RM_OK) return 1;
    if (rm_comm_init_rank(&comm, ctx, n, &sh->id, rank) != RM_OK) {
        std::fprintf(stderr, "rank %d rm_comm_init_rank: %s\n", rank, rm_last_error(ctx));
        return 1;
    }
    uint32_t *frame = nullptr;
    if (rank == 0 && hipMalloc(&frame, (size_t)g_W * g_H * 4) != hipSuccess) return 1;
    rm_stats st{};
    for (int f = 0; f < 2; f++) {
        if (!setup(ctx, kPoses[f])) return 1;
        const rm_status rs = g_runs.empty()
                                 ? rm_render_sharded(comm, g_W, g_H, g_band, frame, rank == 0 ? &st : nullptr)
                                 : rm_render_sharded_runs(comm, g_W, g_H, g_runs.data(), frame, rank == 0 ? &st : nullptr);
        if (rs != RM_OK) {
            std::fprintf(stderr, "rank %d rm_render_sharded: %s\n", rank, rm_last_error(ctx));
            return 1;
        }
        if (rank == 0) {
            std::vector<uint32_t> got((size_t)g_W * g_H), ref;
            if (rm_synchronize(ctx) != RM_OK ||
                hipMemcpy(got.data(), frame, got.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
                !reference(dev, kPoses[f], ref))
                return 1;
            if (got != ref) sh->equal.store(0);
            sh->frames.fetch_add(1);
        }
    }
    if (rank == 0) {
        int uses = 0;
        rm_comm_info(comm, nullptr, nullptr, &uses);
        sh->uses_rccl.store(uses);
        std::snprintf(sh->stats, sizeof(sh->stats), "%s", standin_stats().c_str());
        sh->root_ms[0] = st.kernel_ms;
        sh->root_ms[1] = st.gather_ms;
        sh->root_ms[2] = st.deinterleave_ms;
    }
    rm_comm_destroy(comm);
    if (frame) (void)hipFree(frame);
    rm_destroy(ctx);
    return 0;
}

int run_ranks(int n) {
    auto *sh = static_cast<Shared *>(
        mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
    if (sh == MAP_FAILED) return 1;
    new (sh) Shared();
    sh->equal.store(1);
    std::vector<pid_t> kids;
    for (int r = 0; r < n; r++) {
        pid_t p = fork();
        if (p < 0) return 1;
        if (p == 0) {
            std::fflush(stdout);
            _exit(rank_worker(sh, n, r));
        }
        kids.push_back(p);
    }
    int bad = 0;
    for (pid_t p : kids) {
        int status = 0;
        if (waitpid(p, &status, 0) < 0 || !WIFEXITED(status) || WEXITSTATUS(status) != 0) bad++;
    }
    const bool equal = !bad && sh->equal.load() == 1 && sh->frames.load() == 2;
    std::printf("{\"mode\": \"ranks\", \"n\": %d, \"W\": %d, \"H\": %d, \"band\": %d, \"frames\": %d, \"equal\": %s, "
                "\"failed_ranks\": %d, \"uses_rccl\": %d, \"standin_stats\": %s, \"root_ms\": [%g, %g, %g]}\n",
                n, g_W, g_H, g_band, sh->frames.load(), equal ? "true" : "false", bad, sh->uses_rccl.load(),
                sh->stats[0] ? sh->stats : "null", sh->root_ms[0], sh->root_ms[1], sh->root_ms[2]);
    return equal ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s all|ranks N W H BAND SCENE\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    const int n = std::atoi(argv[2]);
    g_W = std::atoi(argv[3]);
    g_H = std::atoi(argv[4]);
    g_band = std::atoi(argv[5]);
    if (std::strchr(argv[5], ',')) {
        for (const char *q = argv[5]; *q;) {
            g_runs.push_back(std::atoi(q));
            q = std::strchr(q, ',');
            q = q ? q + 1 : "";
        }
        if ((int)g_runs.size() != n) return 2;
        g_band = g_runs[0];
    }
    g_scene = argv[6];
    if (n < 1 || n > 16 || g_W < 1 || g_H < 1 || g_band < 1) return 2;
    if (mode == "all") return run_all(n);
    if (mode == "ranks") return run_ranks(n);
    return 2;
}
