// multi_gpu.cpp — the N-GPU render behind one C-ABI call (gs_render_multi).
//
// Replaces the reference's whole pixel loop, camera.rs:105-114 (pixel list, rayon
// `par_iter` over every pixel, `collect_into_vec`), across the GPUs of one node from a
// single host thread: the scene is uploaded to every device, the frame is cut into
// tiles (cost-balanced plan from a 1-spp pilot on the first device, or round-robin),
// every device renders its tiles into a packed buffer on its own stream, one grouped
// RCCL gather over xGMI brings the packed buffers to the first device, which unpacks
// them into the frame (and, optionally, formats the PPM text, camera.rs:101-103,116-118).
// Pixels carry their own RNG streams, so the frame is the same for any device count.
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

extern "C" void gs_set_last_error(const char* msg);

namespace {

gs_status fail(gs_status code, const std::string& msg) {
    gs_set_last_error(msg.c_str());
    return code;
}

struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
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
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.gather && r.error_string;
        if (!r.ok) r.error = r.path + " lacks ncclCommInitAll/ncclGather";
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

// Everything one call allocates, released on every exit path.
struct Device {
    int id = 0;
    gs_device_scene* scene = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // render start/end, gather start/end
    int32_t* d_order = nullptr;
    float* d_packed = nullptr;
    uint8_t* d_packed8 = nullptr;
    gs_counters* d_cnt = nullptr;
};

struct Job {
    std::vector<Device> dev;
    std::vector<ncclComm_t> comms;
    float *d_gathered = nullptr, *d_frame = nullptr;
    uint8_t *d_gathered8 = nullptr, *d_frame8 = nullptr;
    char* d_text = nullptr;
    void* d_scratch = nullptr;
    int64_t* d_len = nullptr;
    int saved = 0;
    ~Job() {
        for (auto& d : dev) {
            (void)hipSetDevice(d.id);
            if (d.stream) (void)hipStreamSynchronize(d.stream);
        }
        if (!comms.empty() && rccl().ok)
            for (auto c : comms)
                if (c) rccl().comm_destroy(c);
        for (auto& d : dev) {
            (void)hipSetDevice(d.id);
            for (auto e : d.ev)
                if (e) (void)hipEventDestroy(e);
            if (d.d_order) (void)hipFree(d.d_order);
            if (d.d_packed) (void)hipFree(d.d_packed);
            if (d.d_packed8) (void)hipFree(d.d_packed8);
            if (d.d_cnt) (void)hipFree(d.d_cnt);
            if (d.scene) gs_device_scene_destroy(d.scene);
            if (d.stream) (void)hipStreamDestroy(d.stream);
        }
        if (!dev.empty()) {
            (void)hipSetDevice(dev[0].id);
            for (void* p : {(void*)d_gathered, (void*)d_frame, (void*)d_gathered8, (void*)d_frame8, (void*)d_text,
                            d_scratch, (void*)d_len})
                if (p) (void)hipFree(p);
        }
        (void)hipSetDevice(saved);
    }
};

#define HIPOK(x)                                                                                     \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return fail(GS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define ALLOC(p, n)                                                                                           \
    do {                                                                                                      \
        if (hipMalloc((void**)&(p), (size_t)(n) + 16) != hipSuccess)                                         \
            return fail(GS_ERR_OOM, "hipMalloc of " + std::to_string((long long)(n)) + " bytes failed");      \
    } while (0)

}  // namespace

extern "C" {

const char* gs_rccl_library(void) {
    const Rccl& r = rccl();
    return r.ok ? r.path.c_str() : nullptr;
}

gs_status gs_render_multi(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                          const gs_launch* launch, const gs_multi_outputs* out, gs_stats* stats) {
    if (!scene || !cam || !ss || !launch || !out) return fail(GS_ERR_ARG, "null argument");
    if (!out->rgb && !out->rgb8 && !out->ppm_text) return fail(GS_ERR_ARG, "no output requested");
    if (out->ppm_text && !out->ppm_len) return fail(GS_ERR_ARG, "ppm_text without ppm_len");
    if (cam->image_width <= 0 || cam->image_height <= 0) return fail(GS_ERR_ARG, "bad image size");
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) return fail(GS_ERR_NO_DEVICE, "no HIP device visible");
    const int n = launch->num_gpus > 0 ? launch->num_gpus : visible;
    if (n > visible) return fail(GS_ERR_ARG, "num_gpus " + std::to_string(n) + " > visible devices " + std::to_string(visible));
    std::vector<int> ids(n);
    for (int i = 0; i < n; i++) {
        ids[i] = launch->devices ? launch->devices[i] : i;
        if (ids[i] < 0 || ids[i] >= visible) return fail(GS_ERR_ARG, "bad device id");
        for (int j = 0; j < i; j++)
            if (ids[j] == ids[i]) return fail(GS_ERR_ARG, "device listed twice (one communicator rank per device)");
    }
    const int32_t tw = launch->tile_w > 0 ? launch->tile_w : 64, th = launch->tile_h > 0 ? launch->tile_h : tw;
    const int64_t W = cam->image_width, H = cam->image_height;
    const bool want8 = out->rgb8 || out->ppm_text;
    if (out->ppm_text && out->ppm_capacity < gs_ppm_max_bytes(cam->image_width, cam->image_height))
        return fail(GS_ERR_ARG, "ppm_capacity below gs_ppm_max_bytes");
    const Rccl& R = rccl();
    if (!R.ok) return fail(GS_ERR_UNSUPPORTED, "RCCL unavailable: " + R.error);

    const auto t0 = std::chrono::steady_clock::now();
    Job job;
    (void)hipGetDevice(&job.saved);
    job.dev.resize(n);
    for (int i = 0; i < n; i++) {
        Device& d = job.dev[i];
        d.id = ids[i];
        HIPOK(hipSetDevice(d.id));
        const gs_status s = gs_device_scene_create(scene, &d.scene);
        if (s != GS_OK) return s;
        HIPOK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        for (auto& e : d.ev) HIPOK(hipEventCreate(&e));
    }
    // Partition: every rank gets the same packed capacity (rank 0 holds the most tiles).
    std::vector<int32_t> order;
    int32_t slots = 0;
    if (launch->plan && n > 1) {
        HIPOK(hipSetDevice(job.dev[0].id));
        gs_status s = gs_plan_tiles(job.dev[0].scene, cam, seed, n, tw, th, nullptr, 0, &slots);
        if (s != GS_OK) return s;
        order.resize((size_t)slots * n);
        s = gs_plan_tiles(job.dev[0].scene, cam, seed, n, tw, th, order.data(), (int64_t)order.size(), &slots);
        if (s != GS_OK) return s;
    }
    gs_partition p0{0, n, tw, th, nullptr, 0, 0};
    const int64_t cap = order.empty() ? gs_partition_capacity(cam, &p0) : (int64_t)slots * tw * th;
    if (cap < 0) return fail(GS_ERR_ARG, "bad partition");
    const auto t1 = std::chrono::steady_clock::now();

    for (int i = 0; i < n; i++) {
        Device& d = job.dev[i];
        HIPOK(hipSetDevice(d.id));
        if (!order.empty()) {
            ALLOC(d.d_order, order.size() * sizeof(int32_t));
            HIPOK(hipMemcpyAsync(d.d_order, order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                 d.stream));
        }
        if (out->rgb) ALLOC(d.d_packed, cap * 12);
        if (want8) ALLOC(d.d_packed8, cap * 3);
        ALLOC(d.d_cnt, sizeof(gs_counters));
        if (d.d_packed) HIPOK(hipMemsetAsync(d.d_packed, 0, (size_t)cap * 12, d.stream));
        if (d.d_packed8) HIPOK(hipMemsetAsync(d.d_packed8, 0, (size_t)cap * 3, d.stream));
        HIPOK(hipMemsetAsync(d.d_cnt, 0, sizeof(gs_counters), d.stream));
        if (i == 0) {
            if (out->rgb) {
                ALLOC(job.d_gathered, (int64_t)n * cap * 12);
                ALLOC(job.d_frame, W * H * 12);
            }
            if (want8) {
                ALLOC(job.d_gathered8, (int64_t)n * cap * 3);
                ALLOC(job.d_frame8, W * H * 3);
            }
            if (out->ppm_text) {
                ALLOC(job.d_text, gs_ppm_max_bytes(cam->image_width, cam->image_height));
                ALLOC(job.d_scratch, gs_ppm_scratch_bytes(cam->image_width, cam->image_height));
                ALLOC(job.d_len, 8);
            }
        }
    }
    // One communicator rank per device, rank i = device i of the list.
    job.comms.assign(n, nullptr);
    {
        ncclResult_t rc = R.comm_init_all(job.comms.data(), n, ids.data());
        if (rc != ncclSuccess) {
            job.comms.clear();
            return fail(GS_ERR_HIP, std::string("ncclCommInitAll: ") + R.error_string(rc));
        }
    }
    // Render: every device its own tiles, concurrently.
    for (int i = 0; i < n; i++) {
        Device& d = job.dev[i];
        HIPOK(hipSetDevice(d.id));
        gs_partition p{i, n, tw, th, d.d_order, slots, 0};
        gs_render_outputs o{d.d_packed, d.d_packed8, nullptr};
        HIPOK(hipEventRecord(d.ev[0], d.stream));
        const gs_status s = gs_render_tiles_ex_async(d.scene, cam, ss, seed, &p, &o, d.d_cnt, d.stream);
        if (s != GS_OK) return s;
        HIPOK(hipEventRecord(d.ev[1], d.stream));
    }
    // One grouped RCCL gather of the packed tiles to the first device (rank-major, as
    // gs_unpack_tiles_part_async reads them).
    if (R.group_start() != ncclSuccess) return fail(GS_ERR_HIP, "ncclGroupStart failed");
    ncclResult_t rc = ncclSuccess;
    for (int i = 0; i < n && rc == ncclSuccess; i++) {
        Device& d = job.dev[i];
        (void)hipSetDevice(d.id);
        (void)hipEventRecord(d.ev[2], d.stream);
        if (d.d_packed)
            rc = R.gather(d.d_packed, i == 0 ? (void*)job.d_gathered : nullptr, (size_t)cap * 3, ncclFloat32, 0,
                          job.comms[i], d.stream);
        if (rc == ncclSuccess && d.d_packed8)
            rc = R.gather(d.d_packed8, i == 0 ? (void*)job.d_gathered8 : nullptr, (size_t)cap * 3, ncclUint8, 0,
                          job.comms[i], d.stream);
    }
    const ncclResult_t rc2 = R.group_end();
    if (rc != ncclSuccess || rc2 != ncclSuccess)
        return fail(GS_ERR_HIP, std::string("ncclGather: ") + R.error_string(rc != ncclSuccess ? rc : rc2));
    Device& d0 = job.dev[0];
    HIPOK(hipSetDevice(d0.id));
    gs_partition pu{0, n, tw, th, d0.d_order, slots, 0};
    if (out->rgb) {
        const gs_status s = gs_unpack_tiles_part_async(cam, &pu, cap, job.d_gathered, job.d_frame, 12, d0.stream);
        if (s != GS_OK) return s;
    }
    if (want8) {
        const gs_status s = gs_unpack_tiles_part_async(cam, &pu, cap, job.d_gathered8, job.d_frame8, 3, d0.stream);
        if (s != GS_OK) return s;
    }
    HIPOK(hipEventRecord(d0.ev[3], d0.stream));
    if (out->ppm_text) {
        const int64_t need = gs_ppm_max_bytes(cam->image_width, cam->image_height);
        const gs_status s = gs_ppm_encode_async(job.d_frame8, cam->image_width, cam->image_height, job.d_text, need,
                                                job.d_len, job.d_scratch,
                                                gs_ppm_scratch_bytes(cam->image_width, cam->image_height), d0.stream);
        if (s != GS_OK) return s;
    }
    // Results to the host.
    gs_counters total{};
    double rmax = 0.0, rmin = 1e300;
    for (int i = 0; i < n; i++) {
        Device& d = job.dev[i];
        HIPOK(hipSetDevice(d.id));
        HIPOK(hipStreamSynchronize(d.stream));
        gs_counters c{};
        HIPOK(hipMemcpy(&c, d.d_cnt, sizeof(c), hipMemcpyDeviceToHost));
        add_counters(total, c);
        float ms = 0.0f;
        HIPOK(hipEventElapsedTime(&ms, d.ev[0], d.ev[1]));
        rmax = std::max(rmax, (double)ms);
        rmin = std::min(rmin, (double)ms);
    }
    HIPOK(hipSetDevice(d0.id));
    float gms = 0.0f;
    HIPOK(hipEventElapsedTime(&gms, d0.ev[2], d0.ev[3]));
    if (out->rgb) HIPOK(hipMemcpy(out->rgb, job.d_frame, (size_t)(W * H * 12), hipMemcpyDeviceToHost));
    if (out->rgb8) HIPOK(hipMemcpy(out->rgb8, job.d_frame8, (size_t)(W * H * 3), hipMemcpyDeviceToHost));
    if (out->ppm_text) {
        int64_t len = 0;
        HIPOK(hipMemcpy(&len, job.d_len, 8, hipMemcpyDeviceToHost));
        if (len <= 0 || len > out->ppm_capacity) return fail(GS_ERR_HIP, "PPM encoder returned a bad length");
        HIPOK(hipMemcpy(out->ppm_text, job.d_text, (size_t)len, hipMemcpyDeviceToHost));
        *out->ppm_len = len;
    }
    const auto t2 = std::chrono::steady_clock::now();
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->counters = total;
        stats->setup_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats->total_ms = std::chrono::duration<double, std::milli>(t2 - t0).count();
        stats->render_ms_max = rmax;
        stats->render_ms_min = rmin;
        stats->gather_ms = gms;
        stats->algorithmic_bytes = algorithmic_bytes(total);
        stats->gathered_bytes = (uint64_t)n * (uint64_t)cap * ((out->rgb ? 12u : 0u) + (want8 ? 3u : 0u));
        stats->num_gpus = n;
    }
    return GS_OK;
}

}  // extern "C"
