/*
 * grayshift_gpu.h — the C-ABI drop-in boundary of the MI355X path tracer.
 *
 * This is what the reference's `Camera::render` (src/camera.rs:100) calls in place
 * of its pixel loop (camera.rs:105-114: pixel list + rayon `par_iter` + `sample`).
 * The host (the reference's Rust crate, or the C++ mirror in grayshift_amd/csrc/host)
 * builds the world, builds the BVH with the reference's own median split
 * (hittable/BVH.rs:18-65) and flattens it into the plain arrays below; the library
 * copies them into HBM and runs the persistent HIP megakernel.  The output stage
 * (PPM header + write_color, camera.rs:101-103,116-118) stays on the host.
 *
 * Plain pointers and sizes only; no torch, no HIP types in the signatures (a stream
 * is passed as `void*`).  No exceptions cross the ABI: every entry point returns a
 * gs_status and leaves a message for gs_last_error().  Launches of one gs_device_scene
 * may be issued from several host threads and on several streams: each launch takes
 * its own parameter / work-queue / chunk-sum slot from a small ring (a slot is reused
 * only after its previous launch has finished, by a stream wait on that launch's event).
 */
#ifndef GRAYSHIFT_GPU_H
#define GRAYSHIFT_GPU_H

#include <stddef.h>
#include <stdint.h>
#include "grayshift_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 11

typedef int32_t gs_status;
enum {
    GS_OK = 0,
    GS_ERR_ARG = -1,         /* bad argument / malformed scene */
    GS_ERR_HIP = -2,         /* HIP runtime error */
    GS_ERR_OOM = -3,         /* device allocation failed */
    GS_ERR_UNSUPPORTED = -4, /* scene feature the device path does not implement */
    GS_ERR_NO_DEVICE = -5    /* no gfx950 device visible */
};

/* ---- tagged child references (32 bit: kind << 28 | index) ---- */
#define GS_REF_SHIFT 28u
#define GS_REF_MASK 0x0FFFFFFFu
enum gs_ref_kind {
    GS_REF_NONE = 0,     /* absent right child (BVH.rs:20-28 n == 1 wrapper) */
    GS_REF_NODE = 1,     /* BVHNode                       -> nodes[]     */
    GS_REF_SPHERE = 2,   /* stationary Sphere             -> spheres[]   */
    GS_REF_MSPHERE = 3,  /* moving Sphere                 -> mspheres[]  */
    GS_REF_QUAD = 4,     /* Quad                          -> quads[]     */
    GS_REF_TRIANGLE = 5, /* Triangle                      -> triangles[] */
    GS_REF_LIST = 6,     /* HittableList of primitives    -> lists[]     */
    GS_REF_INSTANCE = 7, /* Translate / RotateY           -> instances[] */
    GS_REF_MEDIUM = 8    /* ConstantMedium                -> media[]     */
};
#define GS_MAKE_REF(kind, idx) (((uint32_t)(kind) << GS_REF_SHIFT) | ((uint32_t)(idx) & GS_REF_MASK))

/* BVH node: the reference AABB in f64 (AABB.rs:7-11) and the two children.
 * 64 B = one cache line, array-of-structs: a lane reads its whole node at once. */
typedef struct gs_node {
    double min[3];
    double max[3];
    uint32_t left, right; /* tagged refs; right may be GS_REF_NONE */
    uint32_t pad[2];
} gs_node;

/* Stationary sphere (sphere.rs:11-18): 40 B. */
typedef struct gs_sphere {
    double center[3];
    double radius;
    uint32_t material;
    uint32_t pad;
} gs_sphere;

/* Moving sphere: center(time) = center_start + time * center_path (sphere.rs:51-53). 64 B. */
typedef struct gs_msphere {
    double center_start[3];
    double center_path[3];
    double radius;
    uint32_t material;
    uint32_t pad;
} gs_msphere;

/* Quad with its plane (quad.rs:12-38, plane.rs:10-18): 136 B. */
typedef struct gs_quad {
    double q[3], u[3], v[3], w[3];
    double normal[3];
    double d;
    uint32_t material;
    uint32_t pad;
} gs_quad;

/* Triangle (triangle.rs:10-28): normal = (b-a)x(c-a), unnormalised. 104 B. */
typedef struct gs_triangle {
    double a[3], b[3], c[3];
    double normal[3];
    uint32_t material;
    uint32_t pad;
} gs_triangle;

/* HittableList (hittable.rs:45-91): list_refs[first .. first+count), each a primitive ref. */
typedef struct gs_list {
    uint32_t first, count;
} gs_list;

/* Instance transform, one per Translate / RotateY (hittable.rs:93-215). 32 B.
 * child: the wrapped object (another instance, a list, a primitive, a medium, or a BVH node:
 * a BVH under an instance chain, whose leaves are lists, primitives or media -- not
 * instances; at most 4 instances in a chain).  Other compositions: GS_ERR_UNSUPPORTED. */
enum { GS_INST_TRANSLATE = 1, GS_INST_ROTATE_Y = 2 };
typedef struct gs_instance {
    uint32_t kind;
    uint32_t child;
    double p[3]; /* TRANSLATE: offset; ROTATE_Y: sin_theta, cos_theta, 0 */
} gs_instance;

/* ConstantMedium (hittable/volume.rs:10-29): 16 B.  boundary: an instance chain, a list
 * or a primitive (no BVH, no medium); material: the phase function (any material). */
typedef struct gs_medium {
    uint32_t boundary;
    uint32_t material;
    double density_neg_inv; /* -1 / density (volume.rs:18) */
} gs_medium;

/* Material record (material.rs): 40 B. */
typedef struct gs_material {
    uint32_t kind;    /* gs_mat_kind */
    uint32_t texture; /* LAMBERTIAN / DIFFUSE_LIGHT / ISOTROPIC */
    double albedo[3]; /* METAL */
    double param;     /* METAL: fuzz; DIELECTRIC: refraction_index */
} gs_material;

/* Texture record (texture.rs): 48 B. */
typedef struct gs_texture {
    uint32_t kind;      /* gs_tex_kind */
    uint32_t even, odd; /* CHECKERED: texture indices */
    uint32_t image;     /* IMAGE: index into images[] */
    double color[3];    /* SOLID; NOISE: color[0] = scale (texture.rs:103) */
    double scale_inv;   /* CHECKERED: 1/scale (texture.rs:42) */
} gs_texture;

typedef struct gs_image {
    uint32_t width, height;
    uint64_t offset; /* byte offset into texels8 (RGB8, row-major, top row first) */
} gs_image;

/* Background (camera.rs:246-270).  For HDRI the rotation's matrix entries are
 * precomputed by the host with the exact expressions of rotate_vector (util.rs:67-86). */
typedef struct gs_background {
    uint32_t kind; /* gs_bg_kind */
    uint32_t width, height;
    uint32_t pad;
    double color[3];
    double rot[9]; /* row-major: x' = v.x*rot[0] + v.y*rot[1] + v.z*rot[2], ... */
} gs_background;

/* Flattened scene as handed over by the host. */
typedef struct gs_flat_scene {
    uint32_t root; /* tagged ref of the world BVH root */
    uint32_t max_bvh_depth;
    const gs_node* nodes;         uint32_t n_nodes;
    const gs_sphere* spheres;     uint32_t n_spheres;
    const gs_msphere* mspheres;   uint32_t n_mspheres;
    const gs_quad* quads;         uint32_t n_quads;
    const gs_triangle* triangles; uint32_t n_triangles;
    const gs_list* lists;         uint32_t n_lists;
    const uint32_t* list_refs;    uint32_t n_list_refs;
    const gs_instance* instances; uint32_t n_instances;
    const gs_material* materials; uint32_t n_materials;
    const gs_texture* textures;   uint32_t n_textures;
    const gs_image* images;       uint32_t n_images;
    const uint8_t* texels8;       uint64_t n_texels8;  /* bytes */
    gs_background background;
    const float* hdri_rgb;        uint64_t n_hdri_floats; /* width*height*3 */
    const gs_medium* media;       uint32_t n_media;       /* (ABI 2) */
    /* Perlin::default()'s permutation table (noise 0.9 PermutationTable::new(0)): 256
     * bytes when any texture is NOISE, else NULL / 0 (ABI 3). */
    const uint8_t* noise_perm;    uint32_t n_noise_perm;
} gs_flat_scene;

/* The fields `Camera::new` derives (camera.rs:17-98), computed by the host. */
typedef struct gs_camera {
    int32_t image_width, image_height;
    uint32_t max_depth;
    uint32_t pad;
    double center[3];
    double starting_pixel_pos[3];
    double pixel_delta_u[3];
    double pixel_delta_v[3];
    double defocus_angle;
    double defocus_disk_u[3];
    double defocus_disk_v[3];
} gs_camera;

/* Image-space partition: the frame is cut into tile_w x tile_h tiles.  Position
 * k = slot * world_size + r belongs to rank r; by default position k holds tile k
 * (round-robin, for load balance under adaptive sampling).  A rank's pixels are packed
 * slot after slot, each tile row-major inside, padded to full tiles: packed index =
 * slot*tile_w*tile_h + ty*tile_w + tx.
 * (ABI 3) d_tile_order, when set, is a DEVICE array of slots_per_rank * world_size tile
 * ids, position k -> tile (-1: an empty slot), e.g. the cost-balanced plan of
 * gs_plan_tiles; every tile must appear exactly once. */
typedef struct gs_partition {
    int32_t rank, world_size;
    int32_t tile_w, tile_h;
    const int32_t* d_tile_order; /* nullable */
    int32_t slots_per_rank;      /* with d_tile_order */
    int32_t pad;
} gs_partition;

/* Device-resident scene (opaque): uploaded once, rendered many times. */
typedef struct gs_device_scene gs_device_scene;

const char* gs_last_error(void);
int32_t gs_version(void);

/* Launch tuning, process-wide: shade_batch in [0, 64] = finished lanes a wave
 * collects before it shades them together (0 = the scene's own choice: 52, or 44 for
 * scenes with BVHs under instances; ABI 8); blocks_per_cu in [0, 8], 0 = from the
 * occupancy query; leaf_batch in [0, 64] = lanes waiting at a leaf before the wave
 * runs a leaf-test pass (0 = the scene's own choice: 12, or 48 for scenes with BVHs
 * under instances, whose leaf passes serve one leaf kind each);
 * sample_chunk = samples per work item when the settings run a single batch
 * (max_samples < batch_size, as every fixed-spp render): -1 auto (16, or batch/64 for
 * big batches: at most 64 chunks per pixel, and at most 4 GiB of chunk sums; ABI 7: the
 * launch's last tiles in queue order in the finest chunks, batch/64 or 1, so a frame
 * does not end waiting on a few long items), 0 never split a pixel, n > 0 explicit.
 * Chunks keep every sample's RNG stream; a pixel's chunk sums are added in sample order,
 * so only the association of the f64 colour sum differs from the sequential loop. */
gs_status gs_set_tuning(int32_t shade_batch, int32_t blocks_per_cu, int32_t leaf_batch, int32_t sample_chunk);

/* Node steps per traversal node pass, 1 .. 8 (ABI 4): a node pass lets every lane take
 * up to this many BVH node steps before the wave re-checks which lanes sit at leaves.
 * 0 (default) = the scene's own choice, from its tree's shape at gs_device_scene_create. */
gs_status gs_set_node_steps(int32_t node_steps);

/* Camera-ray batch, process-wide (ABI 9): lanes of a wave that want a camera ray (a new
 * sample's Camera::get_ray, camera.rs:204-221) before the wave generates them together,
 * in [0, 64]; 0 (default) = the scene's own choice.  Waiting lanes idle like finished
 * ones; a wave never waits when none of its lanes has a ray to trace or the work queue
 * is empty.  Every sample's draws and ray are unchanged: only when a lane starts its next
 * sample moves, so frames and counters do not depend on it. */
gs_status gs_set_camera_batch(int32_t cam_batch);

/* Placement of the threaded BVH records (ABI 7).  1 (default): before a scene's first
 * launch, when its records do not all fit the per-block LDS mirror, a pilot renders the
 * launch's camera at 1 spp on a coarse pixel grid counting the tests of every record,
 * and the records are re-placed so the mirror holds the most-tested bytes (the pilot's
 * cost is reported as gs_scene_info.pilot_ms; results never depend on placement).
 * 0: keep the static estimate placed by gs_device_scene_create.  Applies to scenes
 * whose first launch comes after the call.
 * Blocking (ABI 8 note): the launch that runs the pilot waits for it on the host (a
 * stream synchronisation and a copy of the counts) before it issues its own kernels, so
 * that one call of gs_render_tiles*_async is not asynchronous.  A launch of fewer than 16x
 * the pilot's pixel samples (W*H*batch_size < 16 x ~64 k) leaves the pilot to a later,
 * larger launch.  The frame context (gs_multi_render) runs the pilots of all its devices
 * concurrently before its timed render. */
gs_status gs_set_placement(int32_t mode);

/* Diagnostic (ABI 7): one launch like gs_render_tiles_async that also counts, into the
 * device array d_visits (node_records + leaf_records u32, zeroed by the call), the tests
 * of every threaded record by its current position: node records first, then leaf
 * records.  Runs the scene's placement first, like any launch. */
gs_status gs_debug_record_visits(const gs_device_scene* scene, const gs_camera* cam,
                                 const gs_sample_settings* ss, uint64_t seed, const gs_partition* part,
                                 float* d_packed_rgb, uint32_t* d_visits, void* stream);

/* Adaptive settings (ABI 8) -- SampleSettings that run more than one batch
 * (max_samples >= batch_size, camera.rs:135-165).  Batch rounds: round r renders batch r of
 * every pixel still active, its samples spread over the lanes like the fixed-spp chunks,
 * each sample's colour kept; a combine pass then adds each pixel's batch into its running
 * sums in sample order and takes the reference's stop test, so the result is
 * bit-identical to the per-lane loop.  A launch then issues a few small kernels per round
 * on its stream (no host synchronisation).  The per-lane loop: one work item per pixel
 * running all of its batches.  mode 1 (default): rounds when a pixel can take 512 samples
 * or more ((max_samples / batch + 1) x batch: the per-lane loop's tail), else the loop;
 * 2: always rounds; 0: always the loop.  The loop also serves more than 65536 possible
 * batches, a sample chunk of 0 and the diagnostic per-pixel visit output. */
gs_status gs_set_adaptive_mode(int32_t mode);

/* Test hook (ABI 8): the work items of batch rounds.  0 (default): each batch split into
 * sample chunks whose colours a combine pass folds in order.  1: each pixel's batch as one
 * item (from its running sums, the stop test in the lane: no per-sample colours; batches up
 * to 256).  -1: whole-batch items while a round's active pixels are at least twice the
 * device's lanes, split after.  Every choice renders the same bits. */
gs_status gs_debug_set_round_items(int32_t mode);

/* Test hook: scenes uploaded after this call test each Quad::cube list (six consecutive
 * axis-aligned quads in cube order) as straight-line code with the faces' axes fixed at
 * compile time (1, default) or with the generic list loop (0).  Both render the same bits. */
gs_status gs_debug_set_cube_lists(int32_t on);

/* Test hook: the auto sample-chunk rule's budget for chunk sums (default 4 GiB; 0
 * restores it).  A smaller budget makes renders take the chunk-doubling branch. */
gs_status gs_debug_set_partial_budget(uint64_t bytes);

/* Test hook (ABI 10; ABI 11: fine_chunk 0 or 1 only): the auto sample-chunk rule's guided
 * tail -- how much of the frame runs in 1-sample items, as tail_pct percent of the device's
 * lanes x the coarse chunk in samples (0: the default, 200).  tail_pct > 0 also gives an
 * explicit gs_set_tuning sample_chunk (the coarse chunk) a tail.  The tail is scheduling
 * only: its items' sums are regrouped into the coarse chunks, so every choice renders the
 * same bits.  fine_chunk > 1 is rejected (GS_ERR_ARG). */
gs_status gs_debug_set_guided_tail(int32_t fine_chunk, int32_t tail_pct);

/* Upload a flattened scene to the current HIP device. */
gs_status gs_device_scene_create(const gs_flat_scene* scene, gs_device_scene** out);
gs_status gs_device_scene_destroy(gs_device_scene* scene);

/* What gs_device_scene_create built (ABI 5): the threaded top-level tree, the per-block
 * LDS mirror prefixes (before any launch-time shrinking) and the kernel choices taken
 * from the tree's shape.  nodes_per_leaf: expected node tests per leaf test of a ray
 * that enters the root box (surface-area estimate: a record is tested with probability
 * min over its ancestors' box areas / the root box's area); other_leaf_frac: the share of
 * those leaf tests that are not stationary spheres (quads, triangles, lists, instances,
 * media, moving spheres). */
typedef struct gs_scene_info {
    uint32_t node_records, leaf_records;
    uint32_t lds_nodes, lds_leaves, lds_quads;
    int32_t feat;       /* kernel features: 1 media, 2 nested BVHs, 4 sphere leaf runs, 8 whole tree in LDS,
                           64 every top-level leaf a stationary sphere (ABI 7),
                           16 staged shading (three or more shading cases share its stages) */
    int32_t node_steps; /* node steps per node pass the scene's launches use (see gs_set_node_steps) */
    int32_t cert_boxes; /* every node coordinate |x| <= 1e15: the certified f32 box test applies */
    double nodes_per_leaf;
    double other_leaf_frac;
    int32_t placement;  /* (ABI 7) 0 static estimate, first launch pending; 1 static estimate (final);
                           2 measured by the first launch's pilot (gs_set_placement) */
    int32_t long_samples; /* (ABI 11) 1 once a frame of the frame context measured more than 50 lane-us a
                             sample (gs_multi_render's frame notes; sticky): small frames then take the
                             guided tail's 1-sample items too -- scheduling only, the bits are unchanged */
    double pilot_ms;    /* (ABI 7) host time of that pilot and re-placement */
} gs_scene_info;
gs_status gs_device_scene_info(const gs_device_scene* scene, gs_scene_info* out);

/* What one frame did (SURVEY.md §5 metrics row): filled by gs_render, gs_render_ppm,
 * gs_render_multi and gs_multi_render (ABI 6; before ABI 6 only gs_render_multi, and
 * gs_render / gs_render_ppm took a gs_counters*).  Times are HIP events on the launch
 * streams (device) or the host clock (host). */
typedef struct gs_stats {
    gs_counters counters;       /* work done, summed over devices (exact, = the oracle's) */
    double setup_ms;            /* host: scene uploads, communicator and tile plan of this call (one-shot
                                   calls); gs_multi_render: the tile plan when it was (re)computed, plus
                                   the placement pilots of a scene's first frame (ABI 8), else 0 */
    double total_ms;            /* host: the whole call */
    double render_ms_max;       /* slowest device's render: parameter + megakernel + chunk-combine launches */
    double render_ms_min;       /* fastest device's */
    double gather_ms;           /* first device: RCCL gather (N > 1) + unpack (+ PPM text when asked);
                                   one device without a collective renders into the frame itself:
                                   the PPM text's time, else 0 (ABI 10) */
    uint64_t algorithmic_bytes; /* SURVEY.md §8d bytes of every launch (cache-served, not HBM) */
    uint64_t gathered_bytes;    /* bytes the gather delivered to the first device (0 for one device) */
    int32_t num_gpus;
    int32_t pad;
    double kernel_ms_max;       /* (ABI 6) the megakernel alone, slowest device */
    double kernel_ms_min;       /* (ABI 6) the megakernel alone, fastest device */
} gs_stats;

/* Number of packed pixels (tiles * tile_w * tile_h) this rank renders. */
int64_t gs_partition_capacity(const gs_camera* cam, const gs_partition* part);

/* Render this rank's tiles asynchronously on `stream` (hipStream_t as void*, NULL =
 * default stream).  d_packed_rgb: device buffer of capacity*3 f32, linear colour
 * (pixel_color / sample_count, camera.rs:167) for each packed pixel; padding pixels
 * are written as 0.  d_counters: device gs_counters (nullable), accumulated into. */
gs_status gs_render_tiles_async(const gs_device_scene* scene, const gs_camera* cam,
                                const gs_sample_settings* ss, uint64_t seed,
                                const gs_partition* part, float* d_packed_rgb,
                                gs_counters* d_counters, void* stream);

/* Outputs of one launch, per packed pixel (capacity entries; padding pixels get 0).
 * At least one of rgb / rgb8 must be set. */
typedef struct gs_render_outputs {
    float* rgb;            /* capacity*3 f32, linear colour (camera.rs:167), nullable */
    uint8_t* rgb8;         /* capacity*3 u8, write_color's bytes (color.rs:8-18) of the f64
                              colour (not of the f32 one), nullable */
    uint32_t* item_visits; /* capacity u32, BVH node visits per pixel (diagnostic), nullable */
} gs_render_outputs;

/* gs_render_tiles_async with a choice of outputs (ABI 3). */
gs_status gs_render_tiles_ex_async(const gs_device_scene* scene, const gs_camera* cam,
                                   const gs_sample_settings* ss, uint64_t seed,
                                   const gs_partition* part, const gs_render_outputs* out,
                                   gs_counters* d_counters, void* stream);

/* Diagnostic variant: also writes, per packed pixel, the number of BVH node visits
 * its samples made (d_item_visits: capacity u32, nullable; zeroed by the call). */
gs_status gs_render_tiles_debug_async(const gs_device_scene* scene, const gs_camera* cam,
                                      const gs_sample_settings* ss, uint64_t seed,
                                      const gs_partition* part, float* d_packed_rgb,
                                      gs_counters* d_counters, uint32_t* d_item_visits, void* stream);

/* Scatter the packed buffers of all ranks (world_size * capacity * 3 f32, rank-major,
 * as a gather leaves them) into a W*H*3 frame.  Runs on the current device. */
gs_status gs_unpack_tiles_async(const gs_camera* cam, int32_t world_size, int32_t tile_w,
                                int32_t tile_h, int64_t capacity, const float* d_gathered,
                                float* d_frame, void* stream);

/* As gs_unpack_tiles_async, for the 3-byte rgb8 output (ABI 3). */
gs_status gs_unpack_tiles_u8_async(const gs_camera* cam, int32_t world_size, int32_t tile_w,
                                   int32_t tile_h, int64_t capacity, const uint8_t* d_gathered,
                                   uint8_t* d_frame, void* stream);

/* ---- Output stage on the device (camera.rs:101-103,116-118; color.rs:8-18) (ABI 3) ----
 * The reference writes an ASCII PPM: "P3\n{W} {H}\n255\n", then one "{r} {g} {b}\n"
 * line per pixel in row-major order.  gs_ppm_encode_async formats that text on the
 * device from a W*H*3 byte frame (rgb8 output, unpacked): per-block text lengths, one
 * scan into offsets, then each block formats 2048 pixels in LDS and streams them out.
 * The host writes the result with one write call. */
int64_t gs_ppm_max_bytes(int32_t width, int32_t height);     /* text capacity bound */
int64_t gs_ppm_scratch_bytes(int32_t width, int32_t height); /* device scratch size */
/* d_rgb8: device, W*H*3 bytes, 4-byte aligned; d_text: device, >= gs_ppm_max_bytes,
 * 16-byte aligned (hipMalloc'd buffers are); d_len: device
 * int64, receives the text length; d_scratch: device, >= gs_ppm_scratch_bytes, 8-byte
 * aligned (overwritten; reusable once the stream has passed this call). */
gs_status gs_ppm_encode_async(const uint8_t* d_rgb8, int32_t width, int32_t height, char* d_text,
                              int64_t text_capacity, int64_t* d_len, void* d_scratch,
                              int64_t scratch_bytes, void* stream);

/* Synchronous full render to PPM text on the current device: the whole of
 * Camera::render (camera.rs:100-121) past the world build.  out_text: host buffer of
 * text_capacity >= gs_ppm_max_bytes(W, H) bytes; *out_len receives the length. */
gs_status gs_render_ppm(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss,
                        uint64_t seed, char* out_text, int64_t text_capacity, int64_t* out_len,
                        gs_stats* stats /* nullable (ABI 6: was gs_counters*) */);

/* Cost-balanced partition (ABI 3): a 1-spp pilot render of the whole frame on this
 * device (per-pixel BVH node visits, deterministic, so every rank computes the same
 * plan), then longest-processing-time assignment of tiles to world_size ranks (at
 * most ceil(tiles / world_size) each), each rank's tiles in frame order.  Writes
 * order_out (host, world_size * slots entries, see gs_partition.d_tile_order) and
 * *slots_per_rank; order_cap = entries available (query: order_out NULL, returns the
 * entries needed in *slots_per_rank * world_size via *slots_per_rank).  Synchronous. */
gs_status gs_plan_tiles(const gs_device_scene* scene, const gs_camera* cam, uint64_t seed, int32_t world_size,
                        int32_t tile_w, int32_t tile_h, int32_t* order_out, int64_t order_cap,
                        int32_t* slots_per_rank);

/* Unpack for any partition (incl. d_tile_order): elem_bytes 12 (f32 rgb) or 3 (rgb8). */
gs_status gs_unpack_tiles_part_async(const gs_camera* cam, const gs_partition* part, int64_t capacity,
                                     const void* d_gathered, void* d_frame, int32_t elem_bytes, void* stream);

/* ---- The N-GPU render behind one call (ABI 4) ----
 * The whole pixel loop of camera.rs:105-114 on the GPUs of one node, from one host
 * thread: the scene is uploaded to every device, the frame is cut into tile_w x tile_h
 * tiles (plan = 1: cost-balanced, gs_plan_tiles on the first device; 0: round-robin),
 * each device renders its tiles on its own stream, ONE grouped RCCL gather (ncclGather
 * over xGMI, communicator from ncclCommInitAll, one rank per device) brings the packed
 * tiles to the first device, which unpacks them (and formats the PPM text when asked).
 * The frame equals gs_render's for every device count (per-pixel RNG streams).
 * Synchronous; RCCL is loaded at the first call (GS_ERR_UNSUPPORTED without it). */
typedef struct gs_launch {
    int32_t num_gpus;       /* devices used; 0 = every visible device (devices must then be NULL) */
    int32_t tile_w, tile_h; /* 0 = 64 (tile_h 0 = tile_w) */
    int32_t plan;           /* 1: cost-balanced tiles, 0: round-robin */
    const int32_t* devices; /* nullable: num_gpus distinct HIP device ids (default 0..num_gpus-1) */
} gs_launch;

/* Host outputs of gs_render_multi; any subset, at least one. */
typedef struct gs_multi_outputs {
    float* rgb;           /* W*H*3 f32, linear colour (camera.rs:167), nullable */
    uint8_t* rgb8;        /* W*H*3 write_color bytes of the f64 colour, nullable */
    char* ppm_text;       /* the PPM file Camera::render writes (camera.rs:101-118), nullable */
    int64_t ppm_capacity; /* >= gs_ppm_max_bytes(W, H) when ppm_text is set */
    int64_t* ppm_len;     /* receives the text length when ppm_text is set */
} gs_multi_outputs;

gs_status gs_render_multi(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss,
                          uint64_t seed, const gs_launch* launch, const gs_multi_outputs* out, gs_stats* stats);

/* ---- Persistent N-GPU frame context (ABI 6) ----
 * gs_render_multi is gs_multi_create + one gs_multi_render + gs_multi_destroy.  A caller
 * rendering many frames of one world (an animation, a benchmark) creates the context once:
 * the scene upload to every device, the per-device streams and events and the RCCL
 * communicator (ncclCommInitAll, N > 1 only) happen there, outside every frame.  The tile
 * plan is computed at the first frame of a camera and kept while the camera is unchanged.
 * launch->num_gpus <= 0 means every visible device and then requires devices == NULL.
 * num_gpus == 1 uses no collective: the device unpacks its own tiles.
 * A context is not reentrant: one gs_multi_render at a time (calls are serialised). */
typedef struct gs_multi gs_multi;
gs_status gs_multi_create(const gs_flat_scene* scene, const gs_launch* launch, gs_multi** out);
/* One synchronous frame.  out: host outputs (any subset, at least one), or NULL: the linear
 * f32 frame then stays on the first device (gs_multi_frame), nothing crosses PCIe. */
gs_status gs_multi_render(gs_multi* m, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                          const gs_multi_outputs* out, gs_stats* stats);
/* The last frame's device buffers on the first device (W*H*3 f32 / u8; NULL if that output
 * was not produced), valid until the next gs_multi_render or gs_multi_destroy. */
gs_status gs_multi_frame(const gs_multi* m, const float** d_rgb, const uint8_t** d_rgb8, int32_t* device);
/* Devices of the context in rank order (devices: num_gpus entries, nullable). */
gs_status gs_multi_devices(const gs_multi* m, int32_t* num_gpus, int32_t* devices, int32_t capacity);
/* The device-resident scene of rank `rank` (e.g. for gs_device_scene_info); owned by the context. */
gs_status gs_multi_scene(const gs_multi* m, int32_t rank, const gs_device_scene** scene);
gs_status gs_multi_destroy(gs_multi* m);
/* Test hook: 1 = contexts created from now on use the RCCL communicator and gather even for
 * one device (so a one-GPU machine runs that code); 0 (default) = no collective for one. */
gs_status gs_debug_set_multi_collective(int32_t always);
/* Test hook (ABI 11): 1 = contexts created from now on accept a device list that repeats a
 * device (launch->devices) and, for N > 1, gather the ranks' packed tiles by device copies on
 * the ranks' streams instead of RCCL -- so a one-GPU machine runs the N-rank frame loop (one
 * scene, stream and event set per rank, the plan, the concurrent launches, the rank-major
 * unpack, the summed counters, per-rank frame notes) with N scenes on one device; 0 (default). */
gs_status gs_debug_set_multi_same_device(int32_t on);

/* Path of the RCCL library gs_render_multi uses (loaded on this call), or NULL. */
const char* gs_rccl_library(void);

/* Device memory helpers for callers without their own allocator (ctypes, FFI). */
gs_status gs_device_alloc(int64_t bytes, void** d_out);
gs_status gs_device_free(void* d_ptr);
gs_status gs_device_upload(void* d_dst, const void* host_src, int64_t bytes);
gs_status gs_device_download(void* host_dst, const void* d_src, int64_t bytes); /* (ABI 6) synchronous */

/* Synchronous full-frame render on the current device: upload, render, copy back.
 * out_rgb: host buffer W*H*3 f32 (linear).  stats: host, nullable (counters, kernel and
 * render times, algorithmic bytes).  This is the one-call replacement for camera.rs:105-114:
 * gs_multi_create + gs_multi_render + gs_multi_destroy on the current device. */
gs_status gs_render(const gs_flat_scene* scene, const gs_camera* cam, const gs_sample_settings* ss,
                    uint64_t seed, float* out_rgb, gs_stats* stats /* nullable (ABI 6: was gs_counters*) */);

#ifdef __cplusplus
}
#endif
#endif /* GRAYSHIFT_GPU_H */
