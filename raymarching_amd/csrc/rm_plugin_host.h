// rm_plugin_host.h -- host side of scene plugins: hiprtc compilation of a
// scene source into a gfx950 code object, and its module (rm_plugin.h).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "rm_device.h"

namespace rmplugin {

using Code = std::shared_ptr<const std::vector<char>>;

// The GLSL spellings a scene source may use that C++ reads differently,
// rewritten outside comments and literals: unsuffixed floating literals get
// an f (GLSL float, not C++ double); file-scope `const` becomes `constexpr`
// (GLSL constants are usable everywhere, C++ host constants are not usable
// on the device); parameter qualifiers `in` are dropped and `out`/`inout`
// become references; swizzle reads e.xz / e.xyz / e.xyzw become
// swz2/swz3/swz4<indices>(e).  Swizzle writes are not translated.
std::string glsl_source(const std::string& src);

// Compile a (preprocessed) scene source; code objects are cached by source
// text.  On failure `log` holds the compiler's diagnostics.
bool compile(const std::string& src, const std::string& file, Code& code, std::string& log);

struct Module {
    hipModule_t mod = nullptr;
    hipFunction_t render = nullptr;        // timed render kernel; null for an RM_PLUGIN_EVAL_ONLY scene
    hipFunction_t render_count = nullptr;  // instrumented render kernel (ray-step counts, step maps)
    hipFunction_t eval = nullptr;
    Code code;
};
hipError_t load(const Code& code, Module& m);  // on the current device; m keeps its old module on failure
void unload(Module& m);
hipError_t launch_render(const Module& m, const rm::FrameConst& F, void* out, bool rgba8, unsigned long long* evals,
                         hipStream_t s);
hipError_t launch_eval(const Module& m, const rm::FrameConst& F, const float* pts, long long n, float* dist,
                       float* mat, hipStream_t s);

}  // namespace rmplugin
