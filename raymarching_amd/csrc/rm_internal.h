// rm_internal.h -- librm.so-internal accessors of a context (rm_capi.cpp) for
// the other translation units of the library (rm_comm.cpp).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/rm.h"

int rm_internal_device(const rm_ctx *ctx);
hipStream_t rm_internal_stream(const rm_ctx *ctx);
int rm_internal_scene(const rm_ctx *ctx);
// record that work was enqueued on the ctx stream (rm_destroy waits for it)
rm_status rm_internal_mark_done(rm_ctx *ctx);
void rm_internal_set_error(rm_ctx *ctx, const std::string &msg);
