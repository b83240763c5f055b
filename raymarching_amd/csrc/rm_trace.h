// rm_trace.h -- roctx ranges around librm's passes (render, gather, FXAA,
// bloom), so a `rocprofv3 --marker-trace` timeline names them.  The roctx
// library (rocprofiler-sdk) is opened on first use; without it the ranges are
// no-ops.
#pragma once
#include <dlfcn.h>

#include <mutex>

namespace rm {

struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    static const Roctx& get() {
        static Roctx r;
        static std::once_flag once;
        std::call_once(once, [] {
            void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) return;
            r.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
            r.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (!r.push || !r.pop) r.push = nullptr, r.pop = nullptr;
        });
        return r;
    }
};

// RAII range: host-side enqueue span of one pass
class TraceRange {
public:
    explicit TraceRange(const char* name) : on_(Roctx::get().push != nullptr) {
        if (on_) Roctx::get().push(name);
    }
    ~TraceRange() {
        if (on_) Roctx::get().pop();
    }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;

private:
    bool on_;
};

}  // namespace rm
