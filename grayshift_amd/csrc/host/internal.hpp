// internal.hpp — library-internal entry points shared by render.hip and the host files
// (not part of the C-ABI in include/).
#pragma once
#include <hip/hip_runtime_api.h>

#include "../../../include/grayshift_gpu.h"

extern "C" void gs_set_last_error(const char* msg);

// gs_render_tiles_ex_async with two optional timing events (of the stream's device)
// recorded right before and after the megakernel itself, so the frame context can report
// the dominant kernel's time apart from the parameter, queue and chunk-combine launches.
// direct: outs->rgb / rgb8 are the W x H frame itself (image pixel j * W + i; padding slots
// not written), so a one-device frame needs no unpack.  zero_counters: d_counters is set to
// zero by the launch's first kernel instead of accumulated into (no memset before it).
gs_status gs_render_tiles_timed_async(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                      uint64_t seed, const gs_partition* part, const gs_render_outputs* outs,
                                      gs_counters* d_counters, void* stream, hipEvent_t k_begin, hipEvent_t k_end,
                                      bool direct = false, bool zero_counters = false);

// The placement pilots still pending for a launch of `cam` / `ss` on n devices (scenes[i] on
// devices[i], its stream streams[i]): every device's pilot is launched before any is waited
// for, so the first frame of an N-GPU context pilots concurrently (render.hip).  *ran: whether
// any pilot ran.  Leaves the current device changed.
gs_status gs_placement_prepare(gs_device_scene* const* scenes, const int* devices, void* const* streams, int n,
                               const gs_camera* cam, const gs_sample_settings* ss, int* ran);

// A timed frame of the scene on its device: its megakernel time and samples (paths), which
// set the scene's per-sample cost that the guided tail's small-frame rule reads (render.hip).
extern "C" void gs_device_scene_note_frame(gs_device_scene* ds, double kernel_ms, uint64_t samples);
