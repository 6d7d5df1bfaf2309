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
// pixel.  Three launches on the stream, no inter-block waiting: (1) each block of 2048
// pixels sizes its text; (2) one block scans the block lengths into offsets; (3) each
// block formats its text in LDS at the destination's alignment and streams it out in
// 16-byte stores.  (A one-pass decoupled look-back was measured slower here: with every
// block resident at once, only the first blocks hold inclusive prefixes and the walk is
// a chain of cross-XCD load round trips; 87 µs vs this at 4K, see DESIGN.md.)
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
constexpr int SCAN_THREADS = 1024;

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

// A block's pixels: stage their bytes in LDS (coalesced dwords; the host checked 4-byte
// alignment), then each thread sizes the lines of its PPM_PX_PER_THREAD pixels.
struct BlockPixels {
    uint32_t npx, cnt, p_first, mine;
};
__device__ __forceinline__ BlockPixels stage_and_size(const uint8_t* __restrict__ in, uint64_t n_px, uint32_t blk,
                                                      uint32_t* s_in) {
    const uint32_t tid = threadIdx.x;
    BlockPixels b;
    const uint64_t px0 = (uint64_t)blk * PPM_PX;
    b.npx = (uint32_t)((n_px - px0) < (uint64_t)PPM_PX ? (n_px - px0) : (uint64_t)PPM_PX);
    const uint32_t nbytes = b.npx * 3u;
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
    b.p_first = tid * PPM_PX_PER_THREAD;
    b.cnt = b.p_first >= b.npx ? 0u : (b.npx - b.p_first < PPM_PX_PER_THREAD ? b.npx - b.p_first : PPM_PX_PER_THREAD);
    b.mine = 0;
    for (uint32_t k = 0; k < b.cnt; k++) {
        const uint8_t* p = sb + (b.p_first + k) * 3u;
        b.mine += digits(p[0]) + digits(p[1]) + digits(p[2]) + 3u;
    }
    return b;
}

// Block-wide exclusive scan (wave64 shuffles, then across the waves); returns the
// thread's exclusive prefix, *total the block sum.  T: u32 or u64.
template <typename T, int THREADS>
__device__ __forceinline__ T block_scan(T mine, T* s_wave, T* total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    T incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T v = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += v;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    T wave_base = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < THREADS / 64; w++) {
        const T v = s_wave[w];
        if (w < wave) wave_base += v;
        tot += v;
    }
    *total = tot;
    return wave_base + incl - mine;
}

// Pass 1: text length of each block's 2048 pixels.
__global__ __launch_bounds__(PPM_THREADS) void gs_ppm_size_kernel(const uint8_t* __restrict__ in, uint64_t n_px,
                                                                  uint64_t* __restrict__ blk_len) {
    __shared__ uint32_t s_in[PPM_PX * 3 / 4];
    __shared__ uint32_t s_wave[PPM_THREADS / 64];
    const BlockPixels b = stage_and_size(in, n_px, blockIdx.x, s_in);
    uint32_t total;
    block_scan<uint32_t, PPM_THREADS>(b.mine, s_wave, &total);
    if (threadIdx.x == 0) blk_len[blockIdx.x] = total;
}

// Pass 2 (one block): exclusive scan of the block lengths after the header, in place;
// the header text and the total length.
__global__ __launch_bounds__(SCAN_THREADS) void gs_ppm_scan_kernel(uint64_t* __restrict__ blk, uint32_t n_blocks,
                                                                   char* __restrict__ out, int64_t* __restrict__ len_out,
                                                                   PpmHeader hdr) {
    __shared__ uint64_t s_wave[SCAN_THREADS / 64];
    const uint32_t per = (n_blocks + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < n_blocks ? lo + per : n_blocks;
    uint64_t mine = 0;
    for (uint32_t i = lo; i < hi; i++) mine += blk[i];
    uint64_t total;
    uint64_t run = (uint64_t)hdr.len + block_scan<uint64_t, SCAN_THREADS>(mine, s_wave, &total);
    for (uint32_t i = lo; i < hi; i++) {
        const uint64_t v = blk[i];
        blk[i] = run;
        run += v;
    }
    if (threadIdx.x < (uint32_t)hdr.len) out[threadIdx.x] = hdr.c[threadIdx.x];
    if (threadIdx.x == 0) *len_out = (int64_t)(hdr.len + total);
}

// Pass 3: format each block's text in LDS, shifted so that LDS offset and global address
// agree modulo 16, and stream it out in 16-B stores (the two edge chunks, shared with the
// neighbouring blocks, bytewise).
__global__ __launch_bounds__(PPM_THREADS) void gs_ppm_kernel(const uint8_t* __restrict__ in, uint64_t n_px,
                                                             const uint64_t* __restrict__ blk_off,
                                                             char* __restrict__ out) {
    __shared__ uint32_t s_in[PPM_PX * 3 / 4];
    __shared__ __align__(16) uint8_t s_out[PPM_PX * PPM_MAX_LINE + 16];
    __shared__ uint32_t s_wave[PPM_THREADS / 64];
    const BlockPixels b = stage_and_size(in, n_px, blockIdx.x, s_in);
    uint32_t total;
    const uint32_t excl = block_scan<uint32_t, PPM_THREADS>(b.mine, s_wave, &total);
    const uint64_t off = blk_off[blockIdx.x];
    const uint32_t sh = (uint32_t)(off & 15u);
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_in);
    uint32_t at = sh + excl;
    for (uint32_t k = 0; k < b.cnt; k++) {
        const uint8_t* p = sb + (b.p_first + k) * 3u;
        uint8_t* o = s_out + at;
        uint32_t n = put_u8(o, p[0]);
        o[n++] = ' ';
        n += put_u8(o + n, p[1]);
        o[n++] = ' ';
        n += put_u8(o + n, p[2]);
        o[n++] = '\n';
        at += n;
    }
    __syncthreads();
    char* base16 = out + (off - sh);
    const uint32_t end = sh + total;
    const uint32_t nchunks = (end + 15u) >> 4;
    for (uint32_t c = threadIdx.x; c < nchunks; c += PPM_THREADS) {
        const uint32_t lo = c * 16u, hi = lo + 16u;
        if (lo >= sh && hi <= end) {
            *reinterpret_cast<uint4*>(base16 + lo) = *reinterpret_cast<const uint4*>(s_out + lo);
        } else {
            for (uint32_t i = (lo < sh ? sh : lo); i < (hi < end ? hi : end); i++) base16[i] = (char)s_out[i];
        }
    }
}

// Scatter rank-packed tiles into the frame, for any per-pixel element of E bytes (12: f32
// rgb, 3: u8 rgb).  A tile row is one contiguous run in both the packed buffer and the
// frame, so whole V-byte vectors move at once whenever V divides the run, the frame row
// and the tile's x offset (V = 16 for 1080p/4K with 64-px tiles); right-edge padding
// pixels are whole vectors too under that condition, so a vector is stored or skipped.
template <int V>
struct VecOf;
template <>
struct VecOf<16> { using T = uint4; };
template <>
struct VecOf<4> { using T = uint32_t; };
template <>
struct VecOf<1> { using T = uint8_t; };

template <int V>
__global__ void gs_unpack_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ frame, uint32_t E, int32_t W,
                                 int32_t H, int32_t world, int32_t tile_w, int32_t tile_h, int32_t tiles_x,
                                 uint64_t capacity, const int32_t* __restrict__ order) {
    using T = typename VecOf<V>::T;
    const uint64_t run = (uint64_t)tile_w * E;  // bytes per tile row
    const uint64_t rank_bytes = capacity * E;
    const uint64_t units = rank_bytes * (uint64_t)world / V;
    const uint64_t row_bytes = (uint64_t)W * E;
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = u * V;
        const uint32_t r = (uint32_t)(b / rank_bytes);
        const uint64_t rb = b - (uint64_t)r * rank_bytes;
        const uint64_t row = rb / run;  // slot * tile_h + ty
        const uint64_t o = rb - row * run;
        const uint32_t slot = (uint32_t)(row / (uint64_t)tile_h), ty = (uint32_t)(row % (uint64_t)tile_h);
        const uint32_t pos = r + slot * (uint32_t)world;
        const uint32_t tile = order ? (uint32_t)order[pos] : pos;
        if (tile == 0xFFFFFFFFu) continue;  // an empty slot of a planned partition
        const uint64_t x0b = (uint64_t)(tile % (uint32_t)tiles_x) * (uint64_t)tile_w * E;
        const uint32_t y = (tile / (uint32_t)tiles_x) * (uint32_t)tile_h + ty;
        if (y < (uint32_t)H && x0b + o < row_bytes)
            *reinterpret_cast<T*>(frame + (uint64_t)y * row_bytes + x0b + o) = *reinterpret_cast<const T*>(in + b);
    }
}

gs_status unpack(const gs_camera* cam, int32_t world_size, int32_t tile_w, int32_t tile_h, int64_t capacity,
                 const void* d_in, void* d_frame, uint32_t E, void* stream, const int32_t* order = nullptr);

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

gs_status unpack(const gs_camera* cam, int32_t world_size, int32_t tile_w, int32_t tile_h, int64_t capacity,
                 const void* d_in, void* d_frame, uint32_t E, void* stream, const int32_t* order) {
    if (!cam || !d_in || !d_frame || capacity < 0 || world_size < 1 || tile_w < 1 || tile_h < 1 ||
        cam->image_width < 1 || cam->image_height < 1)
        return fail(GS_ERR_ARG, "bad argument");
    if (capacity % ((int64_t)tile_w * tile_h) != 0) return fail(GS_ERR_ARG, "capacity is not whole tiles");
    if (capacity == 0) return GS_OK;
    const int32_t W = cam->image_width, H = cam->image_height;
    const int32_t tiles_x = (W + tile_w - 1) / tile_w;
    auto fits = [&](uint64_t v) {
        return ((uint64_t)W * E) % v == 0 && ((uint64_t)tile_w * E) % v == 0 && ((uintptr_t)d_in % v) == 0 &&
               ((uintptr_t)d_frame % v) == 0;
    };
    const int vec = fits(16) ? 16 : (fits(4) ? 4 : 1);
    const uint64_t units = (uint64_t)capacity * E * (uint64_t)world_size / (uint64_t)vec;
    const unsigned grid = (unsigned)std::min<uint64_t>((units + 255) / 256, 8192);
    hipStream_t st = (hipStream_t)stream;
    const uint8_t* in = (const uint8_t*)d_in;
    uint8_t* fr = (uint8_t*)d_frame;
    if (vec == 16)
        hipLaunchKernelGGL(gs_unpack_kernel<16>, dim3(grid), dim3(256), 0, st, in, fr, E, W, H, world_size, tile_w,
                           tile_h, tiles_x, (uint64_t)capacity, order);
    else if (vec == 4)
        hipLaunchKernelGGL(gs_unpack_kernel<4>, dim3(grid), dim3(256), 0, st, in, fr, E, W, H, world_size, tile_w,
                           tile_h, tiles_x, (uint64_t)capacity, order);
    else
        hipLaunchKernelGGL(gs_unpack_kernel<1>, dim3(grid), dim3(256), 0, st, in, fr, E, W, H, world_size, tile_w,
                           tile_h, tiles_x, (uint64_t)capacity, order);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GS_ERR_HIP, hipGetErrorString(e));
    return GS_OK;
}

}  // namespace

extern "C" {

int64_t gs_ppm_max_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return -1;
    return header_of(width, height, nullptr) + (int64_t)width * height * PPM_MAX_LINE;
}

int64_t gs_ppm_scratch_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return -1;
    return (int64_t)ppm_blocks(width, height) * 8;  // one length / offset per block
}

gs_status gs_ppm_encode_async(const uint8_t* d_rgb8, int32_t width, int32_t height, char* d_text,
                              int64_t text_capacity, int64_t* d_len, void* d_scratch, int64_t scratch_bytes,
                              void* stream) {
    if (!d_rgb8 || !d_text || !d_len || !d_scratch) return fail(GS_ERR_ARG, "null argument");
    if (width <= 0 || height <= 0) return fail(GS_ERR_ARG, "bad image size");
    if ((uint64_t)width * (uint64_t)height >= (1ull << 40)) return fail(GS_ERR_ARG, "image too large");
    if (text_capacity < gs_ppm_max_bytes(width, height)) return fail(GS_ERR_ARG, "text capacity below gs_ppm_max_bytes");
    if (scratch_bytes < gs_ppm_scratch_bytes(width, height)) return fail(GS_ERR_ARG, "scratch below gs_ppm_scratch_bytes");
    if (((uintptr_t)d_rgb8 & 3u) || ((uintptr_t)d_text & 15u) || ((uintptr_t)d_scratch & 7u))
        return fail(GS_ERR_ARG, "rgb8 must be 4-byte aligned, text 16-byte aligned, scratch 8-byte aligned");
    PpmHeader h;
    header_of(width, height, &h);
    const uint32_t nb = ppm_blocks(width, height);
    const uint64_t n_px = (uint64_t)width * (uint64_t)height;
    hipStream_t st = (hipStream_t)stream;
    uint64_t* blk = (uint64_t*)d_scratch;
    hipLaunchKernelGGL(gs_ppm_size_kernel, dim3(nb), dim3(PPM_THREADS), 0, st, d_rgb8, n_px, blk);
    hipLaunchKernelGGL(gs_ppm_scan_kernel, dim3(1), dim3(SCAN_THREADS), 0, st, blk, nb, d_text, d_len, h);
    hipLaunchKernelGGL(gs_ppm_kernel, dim3(nb), dim3(PPM_THREADS), 0, st, d_rgb8, n_px, (const uint64_t*)blk, d_text);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GS_ERR_HIP, hipGetErrorString(e));
    return GS_OK;
}

gs_status gs_unpack_tiles_u8_async(const gs_camera* cam, int32_t world_size, int32_t tile_w, int32_t tile_h,
                                   int64_t capacity, const uint8_t* d_in, uint8_t* d_frame, void* stream) {
    return unpack(cam, world_size, tile_w, tile_h, capacity, d_in, d_frame, 3, stream);
}

gs_status gs_unpack_tiles_part_async(const gs_camera* cam, const gs_partition* part, int64_t capacity,
                                     const void* d_in, void* d_frame, int32_t elem_bytes, void* stream) {
    if (!part || (elem_bytes != 12 && elem_bytes != 3)) return fail(GS_ERR_ARG, "bad argument");
    if (part->d_tile_order && (part->slots_per_rank <= 0 ||
                               capacity != (int64_t)part->slots_per_rank * part->tile_w * part->tile_h))
        return fail(GS_ERR_ARG, "capacity does not match the planned partition");
    return unpack(cam, part->world_size, part->tile_w, part->tile_h, capacity, d_in, d_frame, (uint32_t)elem_bytes,
                  stream, part->d_tile_order);
}

gs_status gs_unpack_tiles_async(const gs_camera* cam, int32_t world_size, int32_t tile_w, int32_t tile_h,
                                int64_t capacity, const float* d_in, float* d_frame, void* stream) {
    return unpack(cam, world_size, tile_w, tile_h, capacity, d_in, d_frame, 12, stream);
}

}  // extern "C"
