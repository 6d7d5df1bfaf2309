// output.hip — the reference's output stage on the device (camera.rs:101-103,116-118;
// color.rs:8-18).
//
// The megakernel can leave write_color's bytes per packed pixel (gs_render_outputs.rgb8,
// computed from the f64 colour exactly as color.rs does).  This file scatters rank-packed
// byte tiles into the frame and formats the frame as the reference's ASCII PPM text:
//
//     "P3\n{W} {H}\n255\n"  then  "{r} {g} {b}\n"  per pixel, row-major
//
// Byte work, HBM-bound (no arithmetic to speak of): 3 B read and 6..12 B written per
// pixel.  One pass: a block formats 2048 pixels in LDS, learns where its text starts by a
// decoupled look-back over its predecessors' lengths (one 8-byte {flag, length} granule
// per block, written and polled with agent-scope atomics, so the hand-off is coherent
// across the 8 XCDs' L2s), then streams its text out with aligned dword stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../../include/grayshift_gpu.h"

extern "C" void gs_set_last_error(const char* msg);

namespace {

constexpr int PPM_THREADS = 256;
constexpr int PPM_PX_PER_THREAD = 8;
constexpr int PPM_PX = PPM_THREADS * PPM_PX_PER_THREAD;  // pixels per block
constexpr int PPM_MAX_LINE = 12;                          // "255 255 255\n"
constexpr uint64_t ST_AGG = 1ull << 62;                   // block's own length is known
constexpr uint64_t ST_INC = 2ull << 62;                   // inclusive prefix is known
constexpr uint64_t ST_VAL = (1ull << 62) - 1;

struct PpmHeader {
    char c[40];
    int32_t len;
};

__device__ __forceinline__ uint32_t digits(uint32_t v) { return 1u + (v >= 10u) + (v >= 100u); }

__device__ __forceinline__ uint32_t put_u8(uint8_t* o, uint32_t v) {
    if (v >= 100u) {
        o[0] = (uint8_t)('0' + v / 100u);
        o[1] = (uint8_t)('0' + (v / 10u) % 10u);
        o[2] = (uint8_t)('0' + v % 10u);
        return 3;
    }
    if (v >= 10u) {
        o[0] = (uint8_t)('0' + v / 10u);
        o[1] = (uint8_t)('0' + v % 10u);
        return 2;
    }
    o[0] = (uint8_t)('0' + v);
    return 1;
}

__global__ __launch_bounds__(PPM_THREADS) void gs_ppm_kernel(const uint8_t* __restrict__ in, uint64_t n_px,
                                                             char* __restrict__ out, int64_t* __restrict__ len_out,
                                                             unsigned long long* __restrict__ status,
                                                             uint32_t* __restrict__ ticket, uint32_t n_blocks,
                                                             PpmHeader hdr) {
    __shared__ uint32_t s_in[PPM_PX * 3 / 4];
    __shared__ uint8_t s_out[PPM_PX * PPM_MAX_LINE];
    __shared__ uint32_t s_wave[PPM_THREADS / 64];
    __shared__ uint32_t s_bid;
    __shared__ unsigned long long s_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    // Dynamic block ids in launch order: a block only ever waits on blocks that already run.
    if (tid == 0) s_bid = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t bid = s_bid;
    const uint64_t px0 = (uint64_t)bid * PPM_PX;
    const uint32_t npx = (uint32_t)((n_px - px0) < (uint64_t)PPM_PX ? (n_px - px0) : (uint64_t)PPM_PX);
    const uint32_t nbytes = npx * 3u;

    // Stage the block's input bytes (coalesced dwords; the host checked 4-byte alignment).
    const uint8_t* src = in + px0 * 3u;
    const uint32_t nfull = nbytes >> 2;
    for (uint32_t i = tid; i < nfull; i += PPM_THREADS) s_in[i] = reinterpret_cast<const uint32_t*>(src)[i];
    if (tid == 0 && (nbytes & 3u)) {
        uint32_t w = 0;
        for (uint32_t k = 0; k < (nbytes & 3u); k++) w |= (uint32_t)src[nfull * 4u + k] << (8u * k);
        s_in[nfull] = w;
    }
    __syncthreads();
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_in);

    // This thread's pixels and their text length.
    const uint32_t p_first = tid * PPM_PX_PER_THREAD;
    const uint32_t cnt = p_first >= npx ? 0u : (npx - p_first < PPM_PX_PER_THREAD ? npx - p_first : PPM_PX_PER_THREAD);
    uint32_t mine = 0;
    for (uint32_t k = 0; k < cnt; k++) {
        const uint8_t* p = sb + (p_first + k) * 3u;
        mine += digits(p[0]) + digits(p[1]) + digits(p[2]) + 3u;
    }
    // Block exclusive scan of the lengths: wave64 shuffles, then across the 4 waves.
    uint32_t incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += v;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t wave_base = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < PPM_THREADS / 64; w++) {
        const uint32_t v = s_wave[w];
        if (w < wave) wave_base += v;
        total += v;
    }
    uint32_t at = wave_base + incl - mine;

    // Format into LDS.
    for (uint32_t k = 0; k < cnt; k++) {
        const uint8_t* p = sb + (p_first + k) * 3u;
        uint8_t* o = s_out + at;
        uint32_t n = put_u8(o, p[0]);
        o[n++] = ' ';
        n += put_u8(o + n, p[1]);
        o[n++] = ' ';
        n += put_u8(o + n, p[2]);
        o[n++] = '\n';
        at += n;
    }

    // Decoupled look-back (one lane): publish this block's length, sum predecessors'
    // lengths back to the first inclusive prefix, publish the inclusive prefix.
    if (tid == 0) {
        uint64_t base;
        if (bid == 0) {
            base = (uint64_t)hdr.len;
        } else {
            __hip_atomic_store(&status[bid], ST_AGG | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            base = 0;
            uint32_t p = bid - 1;
            for (;;) {
                const uint64_t s = __hip_atomic_load(&status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((s & ~ST_VAL) == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                base += s & ST_VAL;
                if ((s & ~ST_VAL) == ST_INC) break;
                p--;  // block 0 always publishes ST_INC, so p never wraps
            }
        }
        __hip_atomic_store(&status[bid], ST_INC | (base + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (bid == n_blocks - 1) *len_out = (int64_t)(base + total);
        s_base = base;
    }
    if (bid == 0 && tid < (uint32_t)hdr.len) out[tid] = hdr.c[tid];
    __syncthreads();

    // Stream the block's text out: byte head up to a dword boundary, dwords, byte tail.
    const uint64_t off = s_base;
    char* dst = out + off;
    const uint32_t head = (uint32_t)((4u - (off & 3u)) & 3u) < total ? (uint32_t)((4u - (off & 3u)) & 3u) : total;
    if (tid < head) dst[tid] = (char)s_out[tid];
    const uint32_t nd = (total - head) >> 2;
    uint32_t* dst32 = reinterpret_cast<uint32_t*>(dst + head);
    for (uint32_t i = tid; i < nd; i += PPM_THREADS) {
        const uint8_t* q = s_out + head + i * 4u;
        dst32[i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    const uint32_t tail = (total - head) & 3u;
    if (tid < tail) dst[head + nd * 4u + tid] = (char)s_out[head + nd * 4u + tid];
}

// Scatter rank-packed byte tiles into the frame (the rgb8 twin of gs_unpack_kernel).
__global__ void gs_unpack_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ frame, int32_t W,
                                    int32_t H, int32_t world, int32_t tile_w, int32_t tile_h, int32_t tiles_x,
                                    uint64_t capacity) {
    const uint64_t total = capacity * (uint64_t)world;
    const uint32_t tile_px = (uint32_t)(tile_w * tile_h);
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(g / capacity);
        const uint64_t k = g % capacity;
        const uint32_t slot = (uint32_t)(k / tile_px), w = (uint32_t)(k % tile_px);
        const uint32_t tile = r + slot * (uint32_t)world;
        const int32_t x = (int32_t)((tile % (uint32_t)tiles_x) * (uint32_t)tile_w + w % (uint32_t)tile_w);
        const int32_t y = (int32_t)((tile / (uint32_t)tiles_x) * (uint32_t)tile_h + w / (uint32_t)tile_w);
        if (x < W && y < H) {
            const size_t o = ((size_t)y * (size_t)W + (size_t)x) * 3;
            frame[o] = in[g * 3];
            frame[o + 1] = in[g * 3 + 1];
            frame[o + 2] = in[g * 3 + 2];
        }
    }
}

gs_status fail(gs_status code, const std::string& msg) {
    gs_set_last_error(msg.c_str());
    return code;
}

int64_t header_of(int32_t W, int32_t H, PpmHeader* h) {
    PpmHeader t{};
    int n = std::snprintf(t.c, sizeof(t.c), "P3\n%d %d\n255\n", (int)W, (int)H);
    t.len = n;
    if (h) *h = t;
    return n;
}

uint32_t ppm_blocks(int32_t W, int32_t H) {
    const uint64_t n = (uint64_t)W * (uint64_t)H;
    return (uint32_t)((n + PPM_PX - 1) / PPM_PX);
}

}  // namespace

extern "C" {

int64_t gs_ppm_max_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return -1;
    return header_of(width, height, nullptr) + (int64_t)width * height * PPM_MAX_LINE;
}

int64_t gs_ppm_scratch_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return -1;
    return 64 + (int64_t)ppm_blocks(width, height) * 8;  // ticket (padded to 64 B) + one status word per block
}

gs_status gs_ppm_encode_async(const uint8_t* d_rgb8, int32_t width, int32_t height, char* d_text,
                              int64_t text_capacity, int64_t* d_len, void* d_scratch, int64_t scratch_bytes,
                              void* stream) {
    if (!d_rgb8 || !d_text || !d_len || !d_scratch) return fail(GS_ERR_ARG, "null argument");
    if (width <= 0 || height <= 0) return fail(GS_ERR_ARG, "bad image size");
    if ((uint64_t)width * (uint64_t)height >= (1ull << 40)) return fail(GS_ERR_ARG, "image too large");
    if (text_capacity < gs_ppm_max_bytes(width, height)) return fail(GS_ERR_ARG, "text capacity below gs_ppm_max_bytes");
    if (scratch_bytes < gs_ppm_scratch_bytes(width, height)) return fail(GS_ERR_ARG, "scratch below gs_ppm_scratch_bytes");
    if (((uintptr_t)d_rgb8 & 3u) || ((uintptr_t)d_text & 3u) || ((uintptr_t)d_scratch & 7u))
        return fail(GS_ERR_ARG, "rgb8 and text must be 4-byte aligned, scratch 8-byte aligned");
    PpmHeader h;
    header_of(width, height, &h);
    const uint32_t nb = ppm_blocks(width, height);
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(d_scratch, 0, (size_t)gs_ppm_scratch_bytes(width, height), st);
    if (e != hipSuccess) return fail(GS_ERR_HIP, hipGetErrorString(e));
    uint32_t* ticket = (uint32_t*)d_scratch;
    unsigned long long* status = (unsigned long long*)((char*)d_scratch + 64);
    hipLaunchKernelGGL(gs_ppm_kernel, dim3(nb), dim3(PPM_THREADS), 0, st, d_rgb8,
                       (uint64_t)width * (uint64_t)height, d_text, d_len, status, ticket, nb, h);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(GS_ERR_HIP, hipGetErrorString(e));
    return GS_OK;
}

gs_status gs_unpack_tiles_u8_async(const gs_camera* cam, int32_t world_size, int32_t tile_w, int32_t tile_h,
                                   int64_t capacity, const uint8_t* d_in, uint8_t* d_frame, void* stream) {
    if (!cam || !d_in || !d_frame || capacity < 0 || world_size < 1 || tile_w < 1 || tile_h < 1 ||
        cam->image_width < 1 || cam->image_height < 1)
        return fail(GS_ERR_ARG, "bad argument");
    if (capacity % ((int64_t)tile_w * tile_h) != 0) return fail(GS_ERR_ARG, "capacity is not whole tiles");
    if (capacity == 0) return GS_OK;
    const int32_t tiles_x = (cam->image_width + tile_w - 1) / tile_w;
    const uint64_t total = (uint64_t)capacity * world_size;
    const unsigned grid = (unsigned)std::min<uint64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(gs_unpack_u8_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_in, d_frame,
                       cam->image_width, cam->image_height, world_size, tile_w, tile_h, tiles_x, (uint64_t)capacity);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GS_ERR_HIP, hipGetErrorString(e));
    return GS_OK;
}

}  // extern "C"
