// rm_plugin_host.cpp -- scene plugins.
//
// The reference reloads its scene by recompiling the preprocessed
// output_shader.frag through sf::Shader::loadFromMemory
// (source/shader_loader.cpp:19; the "Reload scene shader" button,
// main.cpp:134-139).  Here a scene is a source file (".hip") written against
// the reference's scene library (rm_sdf_lib.h, common.frag:37-679):
// rm_load_scene preprocesses it with the reference's #include semantics and
// compiles it with hiprtc for gfx950 into a code object whose kernels are
// output_shader.frag's pass around the scene's sceneSDF (rm_plugin.h,
// rm_plugin_kernels.h).  Code objects are cached per source text, so reloading
// an unchanged scene costs no compilation.
#include "rm_plugin_host.h"

#include <hip/hiprtc.h>

#include <cstdio>
#include <vector>

#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>

extern "C" {
extern const int rm_rtc_header_count;
extern const char* const rm_rtc_header_names[];
extern const char* const rm_rtc_header_texts[];
}

namespace rmplugin {

namespace {

bool is_id(char c) { return std::isalnum((unsigned char)c) || c == '_'; }

// component index of a swizzle letter (xyzw / rgba / stpq), -1 otherwise
int swizzle_index(char c, int set) {
    static const char* sets[3] = {"xyzw", "rgba", "stpq"};
    for (int i = 0; i < 4; i++)
        if (sets[set][i] == c) return i;
    return -1;
}

// "xz" -> "swz2<0, 2>", or "" if w is not a 2-4 letter swizzle of one set
std::string swizzle_call(const std::string& w) {
    if (w.size() < 2 || w.size() > 4) return "";
    for (int set = 0; set < 3; set++) {
        std::string idx;
        bool ok = true;
        for (char c : w) {
            int k = swizzle_index(c, set);
            if (k < 0) {
                ok = false;
                break;
            }
            idx += (idx.empty() ? "" : ", ") + std::to_string(k);
        }
        if (ok) return "swz" + std::to_string(w.size()) + "<" + idx + ">";
    }
    return "";
}

// start (in o) of the postfix expression that ends o: identifiers, member
// chains, and bracketed call / index groups
size_t operand_start(const std::string& o) {
    size_t k = o.size();
    for (;;) {
        if (k > 0 && (o[k - 1] == ')' || o[k - 1] == ']')) {
            const char close = o[k - 1], open = close == ')' ? '(' : '[';
            int depth = 0;
            size_t m = k;
            while (m > 0) {
                m--;
                if (o[m] == close) depth++;
                else if (o[m] == open && --depth == 0) break;
            }
            k = m;
            while (k > 0 && is_id(o[k - 1])) k--;  // a call's or an array's name
        } else if (k > 0 && is_id(o[k - 1])) {
            while (k > 0 && is_id(o[k - 1])) k--;
        } else {
            break;
        }
        if (k > 0 && o[k - 1] == '.') {
            k--;
            continue;
        }
        break;
    }
    return k;
}

}  // namespace

std::string glsl_source(const std::string& s) {
    std::string o;
    o.reserve(s.size() + s.size() / 8);
    const size_t n = s.size();
    size_t i = 0;
    int braces = 0, parens = 0;
    while (i < n) {
        const char c = s[i];
        if (c == '/' && i + 1 < n && (s[i + 1] == '/' || s[i + 1] == '*')) {  // comments
            const bool line = s[i + 1] == '/';
            size_t e = line ? s.find('\n', i) : s.find("*/", i + 2);
            e = e == std::string::npos ? n : (line ? e : e + 2);
            o.append(s, i, e - i);
            i = e;
            continue;
        }
        if (c == '"' || c == '\'') {  // string and character literals
            size_t j = i + 1;
            while (j < n && s[j] != c) j += s[j] == '\\' ? 2 : 1;
            j = j < n ? j + 1 : n;
            o.append(s, i, j - i);
            i = j;
            continue;
        }
        if (std::isalpha((unsigned char)c) || c == '_') {  // identifiers and keywords
            size_t j = i;
            while (j < n && is_id(s[j])) j++;
            const std::string w = s.substr(i, j - i);
            i = j;
            if (w == "const" && braces == 0 && parens == 0) {
                o += "constexpr";
            } else if (parens > 0 && (w == "in" || w == "out" || w == "inout")) {
                while (i < n && (s[i] == ' ' || s[i] == '\t')) i++;
                size_t k = i;
                while (k < n && is_id(s[k])) k++;
                o.append(s, i, k - i);  // the parameter's type
                if (w != "in") o += '&';
                i = k;
            } else {
                o += w;
            }
            continue;
        }
        if (std::isdigit((unsigned char)c) || (c == '.' && i + 1 < n && std::isdigit((unsigned char)s[i + 1]))) {
            size_t j = i + 1;  // a preprocessing number
            while (j < n && (is_id(s[j]) || s[j] == '.' ||
                             ((s[j] == '+' || s[j] == '-') && (s[j - 1] == 'e' || s[j - 1] == 'E'))))
                j++;
            const std::string num = s.substr(i, j - i);
            i = j;
            const bool hex = num.size() > 1 && num[0] == '0' && (num[1] == 'x' || num[1] == 'X');
            o += num;
            if (!hex && num.find_first_of(".eE") != std::string::npos && !std::isalpha((unsigned char)num.back()))
                o += 'f';
            continue;
        }
        if (c == '.' && i + 1 < n && std::isalpha((unsigned char)s[i + 1])) {  // member access or swizzle
            size_t j = i + 1;
            while (j < n && is_id(s[j])) j++;
            const std::string w = s.substr(i + 1, j - i - 1);
            size_t k = j;
            while (k < n && (s[k] == ' ' || s[k] == '\t')) k++;
            const std::string call = swizzle_call(w);
            const bool assigned = k < n && s[k] == '=' && !(k + 1 < n && s[k + 1] == '=');
            if (!call.empty() && !(k < n && s[k] == '(') && !assigned) {
                const size_t a = operand_start(o);
                const std::string operand = o.substr(a);
                o.resize(a);
                o += call + "(" + operand + ")";
                i = j;
                continue;
            }
            o += '.';
            o += w;
            i = j;
            continue;
        }
        if (c == '{') braces++;
        else if (c == '}') braces--;
        else if (c == '(') parens++;
        else if (c == ')') parens--;
        o += c;
        i++;
    }
    return o;
}

namespace {

std::mutex g_mu;
std::map<std::string, Code> g_cache;

std::string translation_unit(const std::string& src, const std::string& file) {
    std::string name;
    for (char c : file) {
        if (c == '"' || c == '\\') name += '\\';
        name += c;
    }
    // the scene twice: against the library's GLSL-rounding instance (rm::glsl:
    // marches, normals, rm_scene_eval) and against its probe instance
    // (rm::glsl::probe, FMA contraction: AO, soft shadows, thickness), as the
    // built-in scenes have exact and probe forms (rm_sdf_lib_body.h)
    const std::string scene = glsl_source(src);
    auto instance = [&](const char* open, const char* close, const char* pre, const char* post) {
        return std::string(open) + "namespace {\n" + pre +
               "#pragma clang force_cuda_host_device begin\n"
               // (every scene function inlined into the kernels: the uniforms are
               // read from the kernel-argument segment, rm_plugin.h; GLSL has no
               // recursion)
               "#pragma clang attribute push (__attribute__((always_inline)), apply_to = function)\n"
               "#line 1 \"" + name + "\"\n" + scene +
               "\n#pragma clang attribute pop\n"
               "#pragma clang force_cuda_host_device end\n" + post + "}  // namespace\n" + close;
    };
    return "#include \"rm_plugin.h\"\n" +
           instance("namespace rm {\nnamespace glsl {\n", "}  // namespace glsl\n}  // namespace rm\n", "", "") +
           instance("namespace rm {\nnamespace glsl {\nnamespace probe {\n",
                    "}  // namespace probe\n}  // namespace glsl\n}  // namespace rm\n",
                    "#pragma clang fp contract(fast)\n#if RM_PROBE_REASSOC\n#pragma clang fp reassociate(on)\n#endif\n",
                    "#if RM_PROBE_REASSOC\n#pragma clang fp reassociate(off)\n#endif\n#pragma clang fp contract(off)\n") +
           "#include \"rm_plugin_kernels.h\"\n";
}

}  // namespace

bool compile(const std::string& src, const std::string& file, Code& code, std::string& log) {
    const std::string tu = translation_unit(src, file);
    log.clear();
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_cache.find(tu);
        if (it != g_cache.end()) {
            code = it->second;
            return true;
        }
    }
    hiprtcProgram prog = nullptr;
    hiprtcResult r = hiprtcCreateProgram(&prog, tu.c_str(), file.c_str(), rm_rtc_header_count, rm_rtc_header_texts,
                                         rm_rtc_header_names);
    if (r != HIPRTC_SUCCESS) {
        log = std::string("hiprtcCreateProgram: ") + hiprtcGetErrorString(r);
        return false;
    }
    // the flags of scene O's translation unit (raymarching_amd/Makefile), no
    // SLP vectorization (as librm's own device code: DEVFLAGS)
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                          "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "-Wno-unused-function",
                          "-Wno-unused-variable"};
    std::vector<const char*> all(opts, opts + sizeof(opts) / sizeof(opts[0]));
    r = hiprtcCompileProgram(prog, (int)all.size(), all.data());
    size_t ls = 0;
    if (hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
        log.resize(ls);
        hiprtcGetProgramLog(prog, &log[0]);
        while (!log.empty() && (log.back() == '\0' || log.back() == '\n')) log.pop_back();
    }
    if (r != HIPRTC_SUCCESS) {
        if (log.empty()) log = hiprtcGetErrorString(r);
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    auto v = std::make_shared<std::vector<char>>(cs);
    hiprtcGetCode(prog, v->data());
    hiprtcDestroyProgram(&prog);
    if (const char* dir = std::getenv("RM_PLUGIN_DUMP")) {  // debugging: the TU and its code object
        std::ofstream(std::string(dir) + "/plugin_tu.hip") << tu;
        std::ofstream(std::string(dir) + "/plugin.co", std::ios::binary).write(v->data(), (std::streamsize)cs);
    }
    code = v;
    std::lock_guard<std::mutex> g(g_mu);
    g_cache[tu] = v;
    return true;
}

hipError_t load(const Code& code, Module& m) {
    Module n;
    hipError_t e = hipModuleLoadData(&n.mod, code->data());
    if (e != hipSuccess) return e;
    if (hipModuleGetFunction(&n.render, n.mod, "rm_plugin_render") != hipSuccess ||
        hipModuleGetFunction(&n.render_count, n.mod, "rm_plugin_render_count") != hipSuccess) {
        (void)hipGetLastError();
        n.render = n.render_count = nullptr;
    }
    e = hipModuleGetFunction(&n.eval, n.mod, "rm_plugin_eval");
    if (e != hipSuccess) {
        (void)hipModuleUnload(n.mod);
        return e;
    }
    n.code = code;
    unload(m);
    m = n;
    return hipSuccess;
}

void unload(Module& m) {
    if (m.mod) (void)hipModuleUnload(m.mod);
    m = Module();
}

hipError_t launch_render(const Module& m, const rm::FrameConst& F, void* out, bool rgba8, unsigned long long* evals,
                         hipStream_t s) {
    if (!m.render || !m.render_count) return hipErrorInvalidDeviceFunction;
    rm::FrameConst f = F;
    f.gx_magic = rm::div_magic((uint32_t)((F.W + 7) / 8), (uint64_t)((F.W + 7) / 8) * (uint64_t)((F.nrows + 7) / 8));
    void* o = out;
    int r8 = rgba8 ? 1 : 0;
    unsigned long long* e = evals;
    void* args[] = {&f, &o, &r8, &e};
    return hipModuleLaunchKernel(evals ? m.render_count : m.render, (unsigned)((F.W + 7) / 8),
                                 (unsigned)((F.nrows + 7) / 8), 1, 64, 1, 1, 0, s, args, nullptr);
}

hipError_t launch_eval(const Module& m, const rm::FrameConst& F, const float* pts, long long n, float* dist,
                       float* mat, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    rm::FrameConst f = F;
    const float* p = pts;
    long long nn = n;
    float* d = dist;
    float* mm = mat;
    void* args[] = {&f, &p, &nn, &d, &mm};
    return hipModuleLaunchKernel(m.eval, (unsigned)((n + 255) / 256), 1, 1, 256, 1, 1, 0, s, args, nullptr);
}

}  // namespace rmplugin
