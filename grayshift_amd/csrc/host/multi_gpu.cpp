// multi_gpu.cpp — the frame context behind the synchronous C-ABI calls: gs_multi_* (one
// world on N GPUs, many frames), and gs_render_multi / gs_render / gs_render_ppm on top.
//
// Replaces the reference's whole pixel loop, camera.rs:105-114 (pixel list, rayon
// `par_iter` over every pixel, `collect_into_vec`), across the GPUs of one node from a
// single host thread: at creation the scene is uploaded to every device and one RCCL
// communicator is built (ncclCommInitAll, N > 1); per frame the image is cut into tiles
// (cost-balanced plan from a 1-spp pilot on the first device, kept while the camera is
// unchanged, or round-robin), every device renders its tiles into a packed buffer on its
// own stream, one grouped RCCL gather over xGMI brings the packed buffers to the first
// device, which unpacks them into the frame (and, optionally, formats the PPM text,
// camera.rs:101-103,116-118).  Pixels carry their own RNG streams, so the frame is the
// same for any device count.
//
// RCCL is resolved at run time (dlopen), so single-GPU users never load it, and the copy
// that matches the process's HIP runtime is used (torch bundles both: one HIP runtime
// per process).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/grayshift_gpu.h"
#include "internal.hpp"

namespace {

gs_status fail(gs_status code, const std::string& msg) {
    gs_set_last_error(msg.c_str());
    return code;
}

struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string path, error;
    bool ok = false;
};

// The RCCL next to the HIP runtime this process uses first (torch/lib/librccl.so beside
// torch's libamdhip64), then the loader's search path, then /opt/rocm.
const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        std::vector<std::string> cands;
        Dl_info info{};
        if (dladdr((const void*)&hipRuntimeGetVersion, &info) && info.dli_fname) {
            std::string dir(info.dli_fname);
            const size_t k = dir.find_last_of('/');
            if (k != std::string::npos) {
                dir.resize(k);
                cands.push_back(dir + "/librccl.so");
                cands.push_back(dir + "/librccl.so.1");
            }
        }
        cands.push_back("librccl.so.1");
        cands.push_back("/opt/rocm/lib/librccl.so.1");
        void* h = nullptr;
        for (const auto& c : cands)
            if ((h = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL)) != nullptr) {
                r.path = c;
                break;
            }
        if (!h) {
            r.error = "librccl not found";
            return;
        }
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.comm_abort = (decltype(r.comm_abort))dlsym(h, "ncclCommAbort");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.ok = r.comm_init_all && r.comm_destroy && r.comm_abort && r.group_start && r.group_end && r.gather &&
               r.error_string;
        if (!r.ok) r.error = r.path + " lacks ncclCommInitAll/ncclCommAbort/ncclGather";
    });
    return r;
}

// SURVEY.md §8d algorithmic bytes per counted event (the same table as bench.py BYTES).
uint64_t algorithmic_bytes(const gs_counters& c) {
    return 56 * c.node_visits + 40 * c.sphere_tests + 64 * c.msphere_tests + 136 * c.quad_tests + 104 * c.tri_tests +
           32 * c.instance_tests + 16 * c.medium_tests + 32 * c.hits + 3 * c.image_texels + 12 * c.hdri_texels +
           12 * c.pixels + 168 * c.noise_evals;
}

void add_counters(gs_counters& a, const gs_counters& b) {
    const uint64_t* pb = (const uint64_t*)&b;
    uint64_t* pa = (uint64_t*)&a;
    for (size_t k = 0; k < sizeof(gs_counters) / sizeof(uint64_t); k++) pa[k] += pb[k];
}

// A device buffer grown on demand (contents not kept).
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool ensure(size_t need) {
        if (bytes >= need && p) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, need + 16) != hipSuccess) return false;
        bytes = need;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct Device {
    int id = 0;
    gs_device_scene* scene = nullptr;
    hipStream_t stream = nullptr;
    // render start / end, megakernel start / end, gather + unpack start / end
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    DBuf order, packed, packed8, cnt;
    // the frame's counters, copied back on the stream behind the frame's last work, so the
    // host's wait is the only synchronisation (a synchronous copy after it cost C1 ~25 us)
    gs_counters* h_cnt = nullptr;  // pinned
};

#define HIPOK(x)                                                                                     \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return fail(GS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define GROW(buf, n)                                                                                            \
    do {                                                                                                        \
        if (!(buf).ensure((size_t)(n)))                                                                         \
            return fail(GS_ERR_OOM, "hipMalloc of " + std::to_string((long long)(n)) + " bytes failed");       \
    } while (0)

// Restores the caller's current device on every exit path.
struct DeviceGuard {
    int saved = 0;
    DeviceGuard() { (void)hipGetDevice(&saved); }
    ~DeviceGuard() { (void)hipSetDevice(saved); }
};

int g_collective_always = 0;  // gs_debug_set_multi_collective
int g_same_device = 0;        // gs_debug_set_multi_same_device

}  // namespace

struct gs_multi {
    std::vector<Device> dev;
    std::vector<int> ids;
    std::vector<ncclComm_t> comms;  // one rank per device (N > 1, or forced by the test hook)
    // gs_debug_set_multi_same_device: N ranks on one device list that may repeat a device, the
    // gather done by device copies on the ranks' streams instead of RCCL (N > 1, no comms)
    bool copy_gather = false;
    bool comms_broken = false;      // a collective failed: the communicators were aborted
    int32_t tw = 64, th = 64;
    bool plan = false;
    mutable std::mutex mu;  // one frame at a time; guards every field below and comms_broken
    // tile partition of the last camera (plan or round-robin)
    bool part_ready = false;
    gs_camera part_cam{};
    std::vector<int32_t> order;  // empty: round-robin
    int32_t slots = 0;
    int64_t cap = 0;  // packed pixels per rank
    // the first device's gather and frame buffers
    DBuf gathered, gathered8, frame, frame8, text, scratch, len;
    bool have_rgb = false, have_rgb8 = false;
    int32_t frame_w = 0, frame_h = 0;

    ~gs_multi() {
        DeviceGuard g;
        if (!comms_broken)
            for (auto& d : dev) {
                (void)hipSetDevice(d.id);
                if (d.stream) (void)hipStreamSynchronize(d.stream);
            }
        if (!comms.empty() && rccl().ok)
            for (auto c : comms)
                if (c) (comms_broken ? rccl().comm_abort(c) : rccl().comm_destroy(c));
        for (auto& d : dev) {
            (void)hipSetDevice(d.id);
            for (auto e : d.ev)
                if (e) (void)hipEventDestroy(e);
            d.order.release();
            d.packed.release();
            d.packed8.release();
            d.cnt.release();
            if (d.h_cnt) (void)hipHostFree(d.h_cnt);
            if (d.scene) gs_device_scene_destroy(d.scene);
            if (d.stream) (void)hipStreamDestroy(d.stream);
        }
        if (!dev.empty()) {
            (void)hipSetDevice(dev[0].id);
            for (DBuf* b : {&gathered, &gathered8, &frame, &frame8, &text, &scratch, &len}) b->release();
        }
    }

    // Abort the communicators after a failed collective: its peers may never join, so the
    // streams holding it must not be waited on (destroy skips the stream syncs).
    gs_status collective_failed(const std::string& what) {
        if (rccl().ok)
            for (auto& c : comms)
                if (c) rccl().comm_abort(c);
        comms.clear();
        comms_broken = true;
        return fail(GS_ERR_HIP, what);
    }

    gs_status partition(const gs_camera* cam, uint64_t seed, double* plan_ms);
    gs_status render(const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed, const gs_multi_outputs* out,
                     gs_stats* stats);
};

gs_status gs_multi::partition(const gs_camera* cam, uint64_t seed, double* plan_ms) {
    if (part_ready && std::memcmp(&part_cam, cam, sizeof(gs_camera)) == 0) return GS_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = (int)dev.size();
    part_ready = false;
    order.clear();
    slots = 0;
    if (plan && n > 1) {
        HIPOK(hipSetDevice(dev[0].id));
        gs_status s = gs_plan_tiles(dev[0].scene, cam, seed, n, tw, th, nullptr, 0, &slots);
        if (s != GS_OK) return s;
        order.resize((size_t)slots * n);
        s = gs_plan_tiles(dev[0].scene, cam, seed, n, tw, th, order.data(), (int64_t)order.size(), &slots);
        if (s != GS_OK) return s;
        for (auto& d : dev) {
            HIPOK(hipSetDevice(d.id));
            GROW(d.order, order.size() * sizeof(int32_t));
            HIPOK(hipMemcpy(d.order.p, order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        }
        cap = (int64_t)slots * tw * th;
    } else {
        gs_partition p0{0, n, tw, th, nullptr, 0, 0};
        cap = gs_partition_capacity(cam, &p0);  // rank 0 holds the most tiles
        if (cap < 0) return fail(GS_ERR_ARG, "bad partition");
    }
    part_cam = *cam;
    part_ready = true;
    *plan_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GS_OK;
}

gs_status gs_multi::render(const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                           const gs_multi_outputs* out, gs_stats* stats) {
    if (!cam || !ss) return fail(GS_ERR_ARG, "null argument");
    if (out && !out->rgb && !out->rgb8 && !out->ppm_text) return fail(GS_ERR_ARG, "no output requested");
    if (out && out->ppm_text && !out->ppm_len) return fail(GS_ERR_ARG, "ppm_text without ppm_len");
    if (cam->image_width <= 0 || cam->image_height <= 0) return fail(GS_ERR_ARG, "bad image size");
    if (out && out->ppm_text && out->ppm_capacity < gs_ppm_max_bytes(cam->image_width, cam->image_height))
        return fail(GS_ERR_ARG, "ppm_capacity below gs_ppm_max_bytes");
    std::lock_guard<std::mutex> lock(mu);
    if (comms_broken) return fail(GS_ERR_HIP, "the context's communicator was aborted after a failed collective");
    DeviceGuard guard;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = (int)dev.size();
    double plan_ms = 0.0;
    gs_status s = partition(cam, seed, &plan_ms);
    if (s != GS_OK) return s;
    {
        // The scenes' placement pilots (first frame, render.hip run before the first launch):
        // launched on every device before any is waited for, outside the timed render.
        std::vector<gs_device_scene*> sc(n);
        std::vector<void*> st(n);
        for (int i = 0; i < n; i++) sc[i] = dev[i].scene, st[i] = dev[i].stream;
        const auto tp = std::chrono::steady_clock::now();
        int ran = 0;
        s = gs_placement_prepare(sc.data(), ids.data(), st.data(), n, cam, ss, &ran);
        if (s != GS_OK) return s;
        if (ran) plan_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
    }
    const bool want_rgb = !out || out->rgb;
    const bool want8 = out && (out->rgb8 || out->ppm_text);
    const int64_t W = cam->image_width, H = cam->image_height;
    have_rgb = have_rgb8 = false;

    // One device and no collective: the render writes the frame itself (no packed tiles,
    // no unpack: C1 saved the unpack kernel and a stream gap, ~20 us of a 0.9 ms frame).
    const bool direct = n == 1 && comms.empty();
    Device& d0 = dev[0];
    HIPOK(hipSetDevice(d0.id));
    if (want_rgb) GROW(frame, W * H * 12);
    if (want8) GROW(frame8, W * H * 3);

    // Render: every device its own tiles, concurrently (launches are asynchronous).
    for (int i = 0; i < n; i++) {
        Device& d = dev[i];
        HIPOK(hipSetDevice(d.id));
        if (want_rgb && !direct) GROW(d.packed, cap * 12);
        if (want8 && !direct) GROW(d.packed8, cap * 3);
        GROW(d.cnt, sizeof(gs_counters));  // (zeroed by the launch's parameter kernel)
        gs_partition p{i, n, tw, th, order.empty() ? nullptr : (const int32_t*)d.order.p, slots, 0};
        gs_render_outputs o{want_rgb ? (float*)(direct ? frame.p : d.packed.p) : nullptr,
                            want8 ? (uint8_t*)(direct ? frame8.p : d.packed8.p) : nullptr, nullptr};
        HIPOK(hipEventRecord(d.ev[0], d.stream));
        s = gs_render_tiles_timed_async(d.scene, cam, ss, seed, &p, &o, (gs_counters*)d.cnt.p, d.stream, d.ev[2],
                                        d.ev[3], direct, true);
        if (s != GS_OK) return s;
        HIPOK(hipEventRecord(d.ev[1], d.stream));
    }
    HIPOK(hipSetDevice(d0.id));
    const void* src = want_rgb ? d0.packed.p : nullptr;
    const void* src8 = want8 ? d0.packed8.p : nullptr;
    if (!comms.empty()) {
        // One grouped RCCL gather of the packed tiles to the first device (rank-major, as
        // gs_unpack_tiles_part_async reads them).
        if (want_rgb) GROW(gathered, (int64_t)n * cap * 12);
        if (want8) GROW(gathered8, (int64_t)n * cap * 3);
        const Rccl& R = rccl();
        for (int i = 0; i < n; i++) {
            HIPOK(hipSetDevice(dev[i].id));
            HIPOK(hipEventRecord(dev[i].ev[4], dev[i].stream));
        }
        if (R.group_start() != ncclSuccess) return collective_failed("ncclGroupStart failed");
        ncclResult_t rc = ncclSuccess;
        for (int i = 0; i < n && rc == ncclSuccess; i++) {
            Device& d = dev[i];
            (void)hipSetDevice(d.id);
            if (want_rgb)
                rc = R.gather(d.packed.p, i == 0 ? gathered.p : nullptr, (size_t)cap * 3, ncclFloat32, 0, comms[i],
                              d.stream);
            if (rc == ncclSuccess && want8)
                rc = R.gather(d.packed8.p, i == 0 ? gathered8.p : nullptr, (size_t)cap * 3, ncclUint8, 0, comms[i],
                              d.stream);
        }
        const ncclResult_t rc2 = R.group_end();
        if (rc != ncclSuccess || rc2 != ncclSuccess)
            return collective_failed(std::string("ncclGather: ") + R.error_string(rc != ncclSuccess ? rc : rc2));
        HIPOK(hipSetDevice(d0.id));
        src = gathered.p;
        src8 = gathered8.p;
    } else if (copy_gather) {
        // The test mode's gather (gs_debug_set_multi_same_device): each rank's packed tiles
        // copied on its own stream into its rank-major slot of the first device's buffer,
        // which ncclGather would fill the same way; the first device's stream waits for all.
        if (want_rgb) GROW(gathered, (int64_t)n * cap * 12);
        if (want8) GROW(gathered8, (int64_t)n * cap * 3);
        for (int i = 0; i < n; i++) {
            Device& d = dev[i];
            HIPOK(hipSetDevice(d.id));
            if (want_rgb)
                HIPOK(hipMemcpyAsync((char*)gathered.p + (size_t)i * cap * 12, d.packed.p, (size_t)cap * 12,
                                     hipMemcpyDeviceToDevice, d.stream));
            if (want8)
                HIPOK(hipMemcpyAsync((char*)gathered8.p + (size_t)i * cap * 3, d.packed8.p, (size_t)cap * 3,
                                     hipMemcpyDeviceToDevice, d.stream));
            HIPOK(hipEventRecord(d.ev[4], d.stream));
        }
        HIPOK(hipSetDevice(d0.id));
        for (int i = 1; i < n; i++) HIPOK(hipStreamWaitEvent(d0.stream, dev[i].ev[4], 0));
        src = gathered.p;
        src8 = gathered8.p;
    }  // (no collective: the unpack is timed from the render's end event, ev[1])
    gs_partition pu{0, n, tw, th, order.empty() ? nullptr : (const int32_t*)d0.order.p, slots, 0};
    if (want_rgb && !direct) {
        s = gs_unpack_tiles_part_async(cam, &pu, cap, src, frame.p, 12, d0.stream);
        if (s != GS_OK) return s;
    }
    if (want8 && !direct) {
        s = gs_unpack_tiles_part_async(cam, &pu, cap, src8, frame8.p, 3, d0.stream);
        if (s != GS_OK) return s;
    }
    if (out && out->ppm_text) {
        const int64_t need = gs_ppm_max_bytes(cam->image_width, cam->image_height);
        const int64_t sb = gs_ppm_scratch_bytes(cam->image_width, cam->image_height);
        GROW(text, need);
        GROW(scratch, sb);
        GROW(len, 8);
        s = gs_ppm_encode_async((const uint8_t*)frame8.p, cam->image_width, cam->image_height, (char*)text.p, need,
                                (int64_t*)len.p, scratch.p, sb, d0.stream);
        if (s != GS_OK) return s;
    }
    // (direct without PPM text: nothing after the render to time, one stream marker fewer)
    const bool timed_tail = !direct || (out && out->ppm_text);
    if (timed_tail) HIPOK(hipEventRecord(d0.ev[5], d0.stream));
    for (auto& d : dev) {
        HIPOK(hipSetDevice(d.id));
        HIPOK(hipMemcpyAsync(d.h_cnt, d.cnt.p, sizeof(gs_counters), hipMemcpyDeviceToHost, d.stream));
    }
    // Wait, then results.
    gs_counters total{};
    double rmax = 0.0, rmin = 1e300, kmax = 0.0, kmin = 1e300;
    for (int i = 0; i < n; i++) {
        Device& d = dev[i];
        HIPOK(hipSetDevice(d.id));
        HIPOK(hipStreamSynchronize(d.stream));
        add_counters(total, *d.h_cnt);
        float ms = 0.0f, kms = 0.0f;
        HIPOK(hipEventElapsedTime(&ms, d.ev[0], d.ev[1]));
        HIPOK(hipEventElapsedTime(&kms, d.ev[2], d.ev[3]));
        gs_device_scene_note_frame(d.scene, (double)kms, d.h_cnt->paths);
        rmax = std::max(rmax, (double)ms);
        rmin = std::min(rmin, (double)ms);
        kmax = std::max(kmax, (double)kms);
        kmin = std::min(kmin, (double)kms);
    }
    HIPOK(hipSetDevice(d0.id));
    float gms = 0.0f;
    if (timed_tail) HIPOK(hipEventElapsedTime(&gms, comms.empty() && !copy_gather ? d0.ev[1] : d0.ev[4], d0.ev[5]));
    have_rgb = want_rgb;
    have_rgb8 = want8;
    frame_w = cam->image_width;
    frame_h = cam->image_height;
    if (out && out->rgb) HIPOK(hipMemcpy(out->rgb, frame.p, (size_t)(W * H * 12), hipMemcpyDeviceToHost));
    if (out && out->rgb8) HIPOK(hipMemcpy(out->rgb8, frame8.p, (size_t)(W * H * 3), hipMemcpyDeviceToHost));
    if (out && out->ppm_text) {
        int64_t l = 0;
        HIPOK(hipMemcpy(&l, len.p, 8, hipMemcpyDeviceToHost));
        if (l <= 0 || l > out->ppm_capacity) return fail(GS_ERR_HIP, "PPM encoder returned a bad length");
        HIPOK(hipMemcpy(out->ppm_text, text.p, (size_t)l, hipMemcpyDeviceToHost));
        *out->ppm_len = l;
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->counters = total;
        stats->setup_ms = plan_ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats->render_ms_max = rmax;
        stats->render_ms_min = rmin;
        stats->kernel_ms_max = kmax;
        stats->kernel_ms_min = kmin;
        stats->gather_ms = gms;
        stats->algorithmic_bytes = algorithmic_bytes(total);
        stats->gathered_bytes =
            comms.empty() && !copy_gather ? 0 : (uint64_t)n * (uint64_t)cap * ((want_rgb ? 12u : 0u) + (want8 ? 3u : 0u));
        stats->num_gpus = n;
    }
    return GS_OK;
}

extern "C" {

const char* gs_rccl_library(void) {
    const Rccl& r = rccl();
    return r.ok ? r.path.c_str() : nullptr;
}

gs_status gs_multi_create(const gs_flat_scene* scene, const gs_launch* launch, gs_multi** out) {
    if (!scene || !launch || !out) return fail(GS_ERR_ARG, "null argument");
    *out = nullptr;
    if (launch->num_gpus <= 0 && launch->devices)
        return fail(GS_ERR_ARG, "num_gpus <= 0 (every visible device) with a device list");
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) return fail(GS_ERR_NO_DEVICE, "no HIP device visible");
    const int n = launch->num_gpus > 0 ? launch->num_gpus : visible;
    if (n > visible && !(g_same_device && launch->devices))  // (the test hook's lists may repeat a device)
        return fail(GS_ERR_ARG, "num_gpus " + std::to_string(n) + " > visible devices " + std::to_string(visible));
    std::vector<int> ids(n);
    for (int i = 0; i < n; i++) {
        ids[i] = launch->devices ? launch->devices[i] : i;
        if (ids[i] < 0 || ids[i] >= visible) return fail(GS_ERR_ARG, "bad device id");
        for (int j = 0; j < i && !g_same_device; j++)
            if (ids[j] == ids[i]) return fail(GS_ERR_ARG, "device listed twice (one communicator rank per device)");
    }
    if (launch->tile_w < 0 || launch->tile_h < 0) return fail(GS_ERR_ARG, "negative tile size");
    const bool copy_gather = g_same_device && n > 1;
    const bool collective = !copy_gather && (n > 1 || g_collective_always);
    if (collective && !rccl().ok) return fail(GS_ERR_UNSUPPORTED, "RCCL unavailable: " + rccl().error);
    DeviceGuard guard;
    auto m = new gs_multi();
    m->ids = ids;
    m->tw = launch->tile_w > 0 ? launch->tile_w : 64;
    m->th = launch->tile_h > 0 ? launch->tile_h : m->tw;
    m->plan = launch->plan != 0;
    m->dev.resize(n);
    m->copy_gather = copy_gather;
    auto bail = [&](gs_status st) {
        delete m;
        return st;
    };
    for (int i = 0; i < n; i++) {
        Device& d = m->dev[i];
        d.id = ids[i];
        if (hipSetDevice(d.id) != hipSuccess) return bail(fail(GS_ERR_HIP, "hipSetDevice failed"));
        const gs_status s = gs_device_scene_create(scene, &d.scene);
        if (s != GS_OK) return bail(s);
        if (hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess)
            return bail(fail(GS_ERR_HIP, "hipStreamCreateWithFlags failed"));
        for (auto& e : d.ev)
            if (hipEventCreate(&e) != hipSuccess) return bail(fail(GS_ERR_HIP, "hipEventCreate failed"));
        if (hipHostMalloc((void**)&d.h_cnt, sizeof(gs_counters), hipHostMallocDefault) != hipSuccess)
            return bail(fail(GS_ERR_OOM, "hipHostMalloc of the counters failed"));
    }
    if (collective) {  // one communicator rank per device, rank i = device i of the list
        m->comms.assign(n, nullptr);
        const ncclResult_t rc = rccl().comm_init_all(m->comms.data(), n, ids.data());
        if (rc != ncclSuccess) {
            m->comms.clear();
            return bail(fail(GS_ERR_HIP, std::string("ncclCommInitAll: ") + rccl().error_string(rc)));
        }
    }
    *out = m;
    return GS_OK;
}

gs_status gs_multi_render(gs_multi* m, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                          const gs_multi_outputs* out, gs_stats* stats) {
    if (!m) return fail(GS_ERR_ARG, "null context");
    return m->render(cam, ss, seed, out, stats);
}

gs_status gs_multi_frame(const gs_multi* m, const float** d_rgb, const uint8_t** d_rgb8, int32_t* device) {
    if (!m) return fail(GS_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lock(m->mu);  // (a frame being rendered replaces these)
    if (d_rgb) *d_rgb = m->have_rgb ? (const float*)m->frame.p : nullptr;
    if (d_rgb8) *d_rgb8 = m->have_rgb8 ? (const uint8_t*)m->frame8.p : nullptr;
    if (device) *device = m->dev[0].id;
    return GS_OK;
}

gs_status gs_multi_devices(const gs_multi* m, int32_t* num_gpus, int32_t* devices, int32_t capacity) {
    if (!m || !num_gpus) return fail(GS_ERR_ARG, "null argument");
    *num_gpus = (int32_t)m->ids.size();
    if (devices)
        for (int32_t i = 0; i < *num_gpus && i < capacity; i++) devices[i] = m->ids[i];
    return GS_OK;
}

gs_status gs_multi_scene(const gs_multi* m, int32_t rank, const gs_device_scene** scene) {
    if (!m || !scene) return fail(GS_ERR_ARG, "null argument");
    if (rank < 0 || rank >= (int32_t)m->dev.size()) return fail(GS_ERR_ARG, "rank out of range");
    *scene = m->dev[rank].scene;
    return GS_OK;
}

gs_status gs_debug_set_multi_collective(int32_t always) {
    g_collective_always = always ? 1 : 0;
    return GS_OK;
}

gs_status gs_debug_set_multi_same_device(int32_t on) {
    if (on != 0 && on != 1) return fail(GS_ERR_ARG, "same-device mode is 0 or 1");
    g_same_device = on;
    return GS_OK;
}

gs_status gs_multi_destroy(gs_multi* m) {
    delete m;
    return GS_OK;
}

gs_status gs_render_multi(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                          const gs_launch* launch, const gs_multi_outputs* out, gs_stats* stats) {
    if (!scene || !cam || !ss || !launch || !out) return fail(GS_ERR_ARG, "null argument");
    const auto t0 = std::chrono::steady_clock::now();
    gs_multi* m = nullptr;
    gs_status s = gs_multi_create(scene, launch, &m);
    if (s != GS_OK) return s;
    const auto t1 = std::chrono::steady_clock::now();
    s = m->render(cam, ss, seed, out, stats);
    gs_multi_destroy(m);
    if (s == GS_OK && stats) {
        stats->setup_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return s;
}

// The one-device, one-frame calls: a context on the current device, no collective.
static gs_status render_here(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss,
                             uint64_t seed, const gs_multi_outputs* out, gs_stats* stats) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(GS_ERR_NO_DEVICE, "no HIP device visible");
    const int32_t ids[1] = {dev};
    gs_launch l{1, 64, 64, 0, ids};
    return gs_render_multi(scene, cam, ss, seed, &l, out, stats);
}

gs_status gs_render(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                    float* out_rgb, gs_stats* stats) {
    if (!scene || !cam || !ss || !out_rgb) return fail(GS_ERR_ARG, "null argument");
    gs_multi_outputs o{out_rgb, nullptr, nullptr, 0, nullptr};
    return render_here(scene, cam, ss, seed, &o, stats);
}

gs_status gs_render_ppm(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                        char* out_text, int64_t text_capacity, int64_t* out_len, gs_stats* stats) {
    if (!scene || !cam || !ss || !out_text || !out_len) return fail(GS_ERR_ARG, "null argument");
    const int64_t need = gs_ppm_max_bytes(cam->image_width, cam->image_height);
    if (need < 0) return fail(GS_ERR_ARG, "bad image size");
    if (text_capacity < need) return fail(GS_ERR_ARG, "text capacity below gs_ppm_max_bytes");
    gs_multi_outputs o{nullptr, nullptr, out_text, text_capacity, out_len};
    return render_here(scene, cam, ss, seed, &o, stats);
}

}  // extern "C"
