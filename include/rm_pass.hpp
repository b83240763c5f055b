// rm_pass.hpp -- C++ host adapter over the rm.h C ABI that mirrors the SFML
// surface the reference's main.cpp drives its ray-march pass through, so that
// main.cpp:52-54,187-207 port one call for one call:
//
//   reference (SFML)                                   here
//   sf::Shader shader;                                 rm::Shader shader(device);
//   ShaderLoader::loadFromFile(f, sf::Shader::Fragment, rm::ShaderLoader::loadFromFile(f, rm::Shader::Fragment,
//                              shader)  -> bool                                    shader) -> bool
//   shader.setUniform("u_pos", sf::Vector3f)           shader.setUniform("u_pos", rm::Vec3{...})
//   sf::RenderTexture t; t.create(w, h);               rm::RenderTexture t; t.create(w, h);
//   t.draw(sprite, &shader);                           t.draw(shader);
//   t.getTexture()                                     t.textureRGBA8() (device RGBA8) / t.copyToHostRGBA8(...)
//
// Errors follow the reference: loadFromFile prints and returns false
// (source/shader_loader.cpp:26-30); other calls return false and keep the
// message in lastError().  Header-only; link with librm.so.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "rm.h"

namespace rm {

struct Vec2 { float x, y; };
struct Vec3 { float x, y, z; };

class Shader {
public:
    enum Type { Fragment };

    explicit Shader(int device = 0) : device_(device) {
        // a librm.so of another ABI would read and write these structs with
        // other layouts (include/rm.h RM_ABI_VERSION)
        if (rm_abi_version() != RM_ABI_VERSION) {
            std::fprintf(stderr, "rm::Shader: librm.so has ABI %d, rm.h declares %d\n", rm_abi_version(),
                         RM_ABI_VERSION);
            return;
        }
        if (rm_create(&ctx_, device) != RM_OK) ctx_ = nullptr;
    }
    ~Shader() {
        if (ctx_) rm_destroy(ctx_);
    }
    Shader(const Shader&) = delete;
    Shader& operator=(const Shader&) = delete;

    bool valid() const { return ctx_ != nullptr; }
    rm_ctx* ctx() { return ctx_; }
    int device() const { return device_; }
    std::string lastError() const { return ctx_ ? rm_last_error(ctx_) : "no HIP device"; }

    bool setUniform(const char* name, float x) { return ctx_ && rm_set_uniform1f(ctx_, name, x) == RM_OK; }
    bool setUniform(const char* name, Vec2 v) { return ctx_ && rm_set_uniform2f(ctx_, name, v.x, v.y) == RM_OK; }
    bool setUniform(const char* name, Vec3 v) {
        return ctx_ && rm_set_uniform3f(ctx_, name, v.x, v.y, v.z) == RM_OK;
    }
    // The reference's compile-time MAX_MARCHING_STEPS (common.frag:15) and the
    // uncapped soft-shadow loop (common.frag:814) are run-time here.
    bool setMarchSteps(int max_steps, int shadow_max_steps = 0) {
        rm_params p;
        if (!ctx_ || rm_get_params(ctx_, &p) != RM_OK) return false;
        p.max_steps = max_steps;
        p.shadow_max_steps = shadow_max_steps;
        return rm_set_params(ctx_, &p) == RM_OK;
    }

private:
    rm_ctx* ctx_ = nullptr;
    int device_ = 0;
};

struct ShaderLoader {
    // source/shader_loader.h:11
    static bool loadFromFile(const char* file_name, Shader::Type, Shader& out_shader) {
        if (!out_shader.valid()) {
            std::fprintf(stderr, "ShaderLoader: no HIP device\n");
            return false;
        }
        return rm_load_scene(out_shader.ctx(), file_name) == RM_OK;  // prints its own message on failure
    }
};

// A W x H render target resident in device memory (sf::RenderTexture).  RGBA8
// by default, the format the reference's RenderTextures hold (main.cpp:34-50):
// the kernel packs the pixel in its epilogue (rm_render_rgba8, 4 B/px of HBM);
// RGBA32F keeps gl_FragColor unrounded (rm_render, 16 B/px).  A draw is
// asynchronous on the shader's stream; copyToHostRGBA8 waits for it.
class RenderTexture {
public:
    enum Format { RGBA8, RGBA32F };

    ~RenderTexture() { release(); }
    bool create(int w, int h, Format fmt = RGBA8) {
        release();
        w_ = w;
        h_ = h;
        fmt_ = fmt;
        return hipMalloc(&tex_, (size_t)w * h * (fmt == RGBA8 ? 4 : 16)) == hipSuccess;
    }
    // RenderTarget::draw(sprite, &shader) with the full-screen sprite (main.cpp:199,205)
    bool draw(Shader& shader, rm_stats* stats = nullptr) {
        if (!tex_) return false;
        return (fmt_ == RGBA8 ? rm_render_rgba8(shader.ctx(), w_, h_, static_cast<uint32_t*>(tex_), stats)
                              : rm_render(shader.ctx(), w_, h_, static_cast<float*>(tex_), stats)) == RM_OK;
    }
    // The same draw reading the ping-pong plumbing (u_sample = this texture,
    // u_sample_part, u_seed1; main.cpp:192-207): progressive accumulation
    // (rm_render_accumulate[_rgba8]).  In place: each pixel reads only itself.
    bool drawAccumulate(Shader& shader, rm_stats* stats = nullptr) {
        if (!tex_) return false;
        return (fmt_ == RGBA8 ? rm_render_accumulate_rgba8(shader.ctx(), w_, h_, static_cast<uint32_t*>(tex_), stats)
                              : rm_render_accumulate(shader.ctx(), w_, h_, static_cast<float*>(tex_), stats)) ==
               RM_OK;
    }
    Format format() const { return fmt_; }
    // the device target: RGBA8 words (R in the low byte) or RGBA32F texels;
    // asking for the other format's view returns null and says so once
    uint32_t* textureRGBA8() { return fmt_ == RGBA8 ? static_cast<uint32_t*>(tex_) : mismatch<uint32_t>("RGBA8"); }
    float* texture() { return fmt_ == RGBA32F ? static_cast<float*>(tex_) : mismatch<float>("RGBA32F"); }
    int width() const { return w_; }
    int height() const { return h_; }
    // RGBA8 (the reference target's format), row 0 first (looks up).  An
    // RGBA32F target is packed into a device buffer kept for later calls.
    bool copyToHostRGBA8(Shader& shader, std::vector<uint32_t>& out) {
        out.resize((size_t)w_ * h_);
        const uint32_t* src = textureRGBA8();
        if (!src) {
            if (!packed_ && hipMalloc(&packed_, out.size() * sizeof(uint32_t)) != hipSuccess) {
                packed_ = nullptr;
                return false;
            }
            if (rm_pack_rgba8(shader.ctx(), (int64_t)out.size(), static_cast<const float*>(tex_), packed_) != RM_OK)
                return false;
            src = packed_;
        }
        return rm_synchronize(shader.ctx()) == RM_OK &&
               hipMemcpy(out.data(), src, out.size() * sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess;
    }

private:
    template <typename T>
    T* mismatch(const char* want) {
        if (!warned_) {
            std::fprintf(stderr, "rm::RenderTexture: a %s view of a %s target (create(w, h, RenderTexture::%s))\n",
                         want, fmt_ == RGBA8 ? "RGBA8" : "RGBA32F", want);
            warned_ = true;
        }
        return nullptr;
    }
    void release() {
        if (tex_) (void)hipFree(tex_);
        if (packed_) (void)hipFree(packed_);
        tex_ = nullptr;
        packed_ = nullptr;
    }
    void* tex_ = nullptr;
    uint32_t* packed_ = nullptr;
    int w_ = 0, h_ = 0;
    Format fmt_ = RGBA8;
    bool warned_ = false;
};

// The multi-GPU form of RenderTexture::draw: a W x H RGBA8 frame whose row
// bands are rendered by one Shader per GPU and gathered over RCCL to the first
// shader's device (rm_comm_init_all + rm_render_sharded_all, one process
// driving N GPUs).  Set the same uniforms on every shader before draw().
class ShardedRenderTexture {
public:
    ~ShardedRenderTexture() { release(); }
    bool create(int w, int h, const std::vector<Shader*>& shaders, int band = 16) {
        release();
        if (shaders.empty()) return false;
        std::vector<rm_ctx*> ctxs;
        for (Shader* s : shaders) {
            if (!s || !s->valid()) return false;
            ctxs.push_back(s->ctx());
        }
        comms_.assign(ctxs.size(), nullptr);
        if (rm_comm_init_all(comms_.data(), ctxs.data(), (int)ctxs.size()) != RM_OK) {
            comms_.clear();
            return false;
        }
        root_ = shaders[0];
        w_ = w;
        h_ = h;
        band_ = band;
        int dev = 0;
        (void)hipGetDevice(&dev);
        bool ok = hipSetDevice(root_->device()) == hipSuccess &&
                  hipMalloc(&frame_, (size_t)w * h * sizeof(uint32_t)) == hipSuccess;
        (void)hipSetDevice(dev);
        return ok;
    }
    // stats: one rm_stats per GPU (or null)
    bool draw(rm_stats* stats = nullptr) {
        return frame_ && rm_render_sharded_all(comms_.data(), (int)comms_.size(), w_, h_, band_, frame_, stats) == RM_OK;
    }
    uint32_t* frame() { return frame_; }
    bool copyToHostRGBA8(std::vector<uint32_t>& out) {
        out.resize((size_t)w_ * h_);
        return rm_synchronize(root_->ctx()) == RM_OK && hipSetDevice(root_->device()) == hipSuccess &&
               hipMemcpy(out.data(), frame_, out.size() * sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess;
    }

private:
    void release() {
        for (rm_comm* c : comms_)
            if (c) rm_comm_destroy(c);
        comms_.clear();
        if (frame_) (void)hipFree(frame_);
        frame_ = nullptr;
    }
    std::vector<rm_comm*> comms_;
    Shader* root_ = nullptr;
    uint32_t* frame_ = nullptr;
    int w_ = 0, h_ = 0, band_ = 16;
};

}  // namespace rm
