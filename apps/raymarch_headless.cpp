// raymarch_headless.cpp -- the reference's frame loop (main.cpp:12-226)
// without a window: the ray-march pass runs through rm::Shader /
// rm::RenderTexture (include/rm_pass.hpp -> librm.so) exactly where main.cpp
// calls ShaderLoader / sf::Shader::setUniform / RenderTexture::draw.
//
// Input comes from a script instead of SFML events: one character per frame,
// W/A/S/D/U(p)/N(down) move as the reference's WASD/Space/LShift
// (main.cpp:111-126,155-171), '.' = no key; --mouse dx,dy adds a per-frame
// mouse delta (main.cpp:86-97).  The FXAA/bloom passes and the ImGui overlay
// stay out of scope (they remain on the reference's GL path).
//
// Usage: raymarch_headless [--scene output_shader.frag] [--w 1600] [--h 900]
//          [--frames 60] [--script WWWWDD..] [--mouse 3,0] [--time-freeze]
//          [--steps 128] [--ppm out.ppm] [--gpus N] [--band 16] [--accumulate]
//          [--format rgba8|float] [--stats] [--warmup N]
// Frames are drawn into the RGBA8 target the reference renders into
// (--format float: RGBA32F) and queued without a host synchronization per
// frame; --stats times each frame's kernel (HIP events, which waits for every
// frame) and reports kernel_ms_per_frame.  fps_wall counts the frames after
// --warmup (untimed) frames, up to the completion of the last one.
// --gpus N renders each frame's row bands on GPUs 0..N-1 and gathers them over
// RCCL to GPU 0 (rm::ShardedRenderTexture -> rm_render_sharded_all); --sharded
// takes that path with one GPU too.
#include <chrono>
#include <cmath>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/rm_pass.hpp"

int main(int argc, char** argv) {
    std::string scene = "output_shader.frag", script, ppm;
    int w = 1600, h = 900, frames = 60, steps = 128, gpus = 1, band = 16;
    int mdx = 0, mdy = 0;
    bool time_freeze = false, sharded = false, accumulate = false, stats = false, fmt_float = false;
    int warmup = 0;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
        if (a == "--scene") scene = next();
        else if (a == "--w") w = std::atoi(next().c_str());
        else if (a == "--h") h = std::atoi(next().c_str());
        else if (a == "--frames") frames = std::atoi(next().c_str());
        else if (a == "--script") script = next();
        else if (a == "--steps") steps = std::atoi(next().c_str());
        else if (a == "--gpus") gpus = std::atoi(next().c_str());
        else if (a == "--band") band = std::atoi(next().c_str());
        else if (a == "--ppm") ppm = next();
        else if (a == "--time-freeze") time_freeze = true;
        else if (a == "--sharded") sharded = true;
        else if (a == "--accumulate") accumulate = true;
        else if (a == "--stats") stats = true;
        else if (a == "--warmup") warmup = std::atoi(next().c_str());
        else if (a == "--format") {
            const std::string f = next();
            if (f != "rgba8" && f != "float") {
                std::fprintf(stderr, "--format rgba8|float\n");
                return 2;
            }
            fmt_float = f == "float";
        }
        else if (a == "--mouse") std::sscanf(next().c_str(), "%d,%d", &mdx, &mdy);
        else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    // main.cpp:14-27
    float wf = (float)w, hf = (float)h;
    int mouseX = w / 2, mouseY = h / 2;
    const float mouseSensitivity = 3.0f, speed = 0.1f;
    rm::Vec3 pos{2.0f, 3.0f, 3.0f};
    int framesStill = 1;

    if (gpus < 1) {
        std::fprintf(stderr, "--gpus must be >= 1\n");
        return 2;
    }
    if (accumulate && (gpus > 1 || sharded)) {
        std::fprintf(stderr, "--accumulate renders on one GPU\n");
        return 2;
    }
    // one shader (librm context) per GPU; the first is the reference's `shader`
    std::vector<std::unique_ptr<rm::Shader>> shaders;
    std::vector<rm::Shader*> all;
    for (int g = 0; g < gpus; g++) {
        shaders.emplace_back(new rm::Shader(g));
        rm::Shader& s = *shaders.back();
        if (!s.valid()) {
            std::fprintf(stderr, "no HIP device %d\n", g);
            return 1;
        }
        if (!rm::ShaderLoader::loadFromFile(scene.c_str(), rm::Shader::Fragment, s)) return 1;
        s.setUniform("u_resolution", rm::Vec2{wf, hf});
        s.setMarchSteps(steps);
        all.push_back(&s);
    }
    rm::Shader& shader = *all[0];
    sharded = sharded || gpus > 1;
    auto setAll = [&](const char* name, auto v) {
        for (rm::Shader* s : all) s->setUniform(name, v);
    };
    rm::RenderTexture outputTexture;
    rm::ShardedRenderTexture shardedTexture;
    if (!sharded ? !outputTexture.create(w, h, fmt_float ? rm::RenderTexture::RGBA32F : rm::RenderTexture::RGBA8)
                 : !shardedTexture.create(w, h, all, band)) {
        std::fprintf(stderr, "cannot allocate the %dx%d target on %d GPU(s): %s\n", w, h, gpus,
                     shader.lastError().c_str());
        return 1;
    }

    std::mt19937 e2(20261015);
    std::uniform_real_distribution<float> dist(0.0f, 1.0f);
    auto t0 = std::chrono::steady_clock::now();
    auto t_timed = t0;
    double kernel_ms = 0.0;
    for (int f = 0; f < warmup + frames; f++) {
        if (f == warmup) {  // the timed frames start when the warm-up frames are done
            if (rm_synchronize(shader.ctx()) != RM_OK) return 1;
            t_timed = std::chrono::steady_clock::now();
        }
        bool wasd[6] = {false, false, false, false, false, false};
        char k = f < (int)script.size() ? script[f] : '.';
        const char keys[] = "WASDUN";
        for (int j = 0; j < 6; j++) wasd[j] = (k == keys[j]);
        mouseX += mdx;
        mouseY += mdy;
        if (mdx || mdy) framesStill = 1;
        // main.cpp:153-171: camera angles and a step along the view-rotated axes
        float mx = ((float)mouseX / w - 0.5f) * mouseSensitivity;
        float my = ((float)mouseY / h - 0.5f) * mouseSensitivity;
        float dx = (float)(wasd[3] - wasd[1]), dy = (float)(wasd[4] - wasd[5]), dz = (float)(wasd[2] - wasd[0]);
        float ty = dy * std::cos(-my) - dz * std::sin(-my);
        float tz = dy * std::sin(-my) + dz * std::cos(-my);
        float tx = dx;
        float nx = tx * std::cos(mx) - tz * std::sin(mx);
        float nz = tx * std::sin(mx) + tz * std::cos(mx);
        pos = rm::Vec3{pos.x + nx * speed, pos.y + ty * speed, pos.z + nz * speed};
        for (bool b : wasd)
            if (b) framesStill = 1;
        setAll("u_pos", pos);
        setAll("u_mouse", rm::Vec2{mx, my});
        if (!time_freeze) {
            float t = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
            setAll("u_time", t);
        }
        setAll("u_sample_part", 1.0f / framesStill);
        const rm::Vec2 seed1{dist(e2) * 999.0f, dist(e2) * 999.0f}, seed2{dist(e2) * 999.0f, dist(e2) * 999.0f};
        setAll("u_seed1", seed1);
        setAll("u_seed2", seed2);
        std::vector<rm_stats> st(gpus);
        rm_stats* stp = stats ? st.data() : nullptr;
        // --accumulate: the pass reads u_sample/u_sample_part/u_seed1 (progressive
        // supersampling while the camera is still; one GPU)
        const bool drawn = sharded      ? shardedTexture.draw(stp)
                           : accumulate ? outputTexture.drawAccumulate(shader, stp)
                                        : outputTexture.draw(shader, stp);
        if (!drawn) {
            std::fprintf(stderr, "draw failed: %s\n", shader.lastError().c_str());
            return 1;
        }
        float slowest = 0.0f;
        for (const rm_stats& x : st) slowest = x.kernel_ms > slowest ? x.kernel_ms : slowest;
        if (f >= warmup) kernel_ms += slowest;
        framesStill++;
    }
    for (rm::Shader* s : all)
        if (rm_synchronize(s->ctx()) != RM_OK) return 1;
    double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_timed).count();
    std::printf("{\"frames\": %d, \"warmup\": %d, \"w\": %d, \"h\": %d, \"gpus\": %d, \"scene\": \"%s\", "
                "\"format\": \"%s\", \"fps_wall\": %.2f, ",
                frames, warmup, w, h, gpus, scene.c_str(), sharded || !fmt_float ? "rgba8" : "float", frames / wall);
    if (stats) std::printf("\"kernel_ms_per_frame\": %.4f, ", frames ? kernel_ms / frames : 0.0);
    std::printf("\"pos\": [%.4f, %.4f, %.4f]}\n", pos.x, pos.y, pos.z);
    if (!ppm.empty()) {
        std::vector<uint32_t> px;
        if (!sharded ? !outputTexture.copyToHostRGBA8(shader, px) : !shardedTexture.copyToHostRGBA8(px)) return 1;
        FILE* fp = std::fopen(ppm.c_str(), "wb");
        if (!fp) return 1;
        std::fprintf(fp, "P6\n%d %d\n255\n", w, h);
        for (uint32_t v : px) {
            unsigned char rgb[3] = {(unsigned char)(v & 255), (unsigned char)((v >> 8) & 255),
                                    (unsigned char)((v >> 16) & 255)};
            std::fwrite(rgb, 1, 3, fp);
        }
        std::fclose(fp);
    }
    return 0;
}
