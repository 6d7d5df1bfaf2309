// render.hip — persistent-wavefront path-tracing megakernel for gfx950 (MI355X),
// and the device half of the C-ABI in include/grayshift_gpu.h.
//
// What it replaces: the reference's per-pixel loop camera.rs:105-114 →
// Camera::sample (camera.rs:125-171) → recursive Camera::ray_color (:174-202) →
// BVHNode::hit (BVH.rs:69-90) / AABB::hit (AABB.rs:58-113) / primitive hits →
// Material::scatter (material.rs) → Texture::value_at / HDRI::sample.
//
// Structure:
//  * a lane owns one work item — a pixel, or for single-batch settings a chunk of one
//    pixel's consecutive samples — and runs its samples in the reference's order, so
//    the per-pixel sums accumulate exactly as camera.rs:138-147 does (chunk sums are
//    added in order by gs_combine_kernel);
//  * a wave hands finished lanes items from its private reserve, refilled by one
//    atomicAdd of up to 32 items on the global queue, so sky pixels never wait for
//    busy ones;
//  * each lane runs a small state machine NEED → TRACE → SHADE → (TRACE | NEED):
//    the wave keeps stepping BVH traversal until `shade_batch` lanes have finished
//    their ray, then shades those lanes together (active-ray packing) while the
//    others keep their traversal state (one record index) for the next round;
//  * traversal is the reference's left-first DFS with a global closest-t, restated
//    over the tree's pre-order records with hit/miss links (no stack), identical in
//    node visits and primitive tests; the most-tested records are mirrored in LDS;
//  * the hit record is recomputed once per ray from (primitive, t) after traversal,
//    which yields the same values the reference computes at every accepted hit.
// All arithmetic is f64 with -ffp-contract=off, as the reference's Rust.

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cmath>
#include <cstring>
#include <atomic>
#include <chrono>
#include <functional>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../../include/grayshift_gpu.h"
#include "../host/internal.hpp"
#include "devmath.hpp"
#include "geometry.hpp"
#include "perlin.hpp"

using namespace gsd;

// One 1024-lane block per CU (4 waves/SIMD): the block's LDS holds the lane state and
// the largest mirror of the tree's top records (1456 of them; measured on MI355X C4:
// 256-lane blocks with 352 mirrored records 4060, 1024-lane blocks 4150 Msamples/s).
#ifndef GS_BLOCK
#define GS_BLOCK 1024
#endif
// Measured on MI355X (C4): everything inlined with a 4-waves/SIMD register cap (128
// VGPRs; spills only in shading) beats out-of-line shading calls and 3 or 5 waves.
#ifndef GS_NOINLINE
#define GS_NOINLINE __forceinline__
#endif
#ifndef GS_MIN_WAVES
#define GS_MIN_WAVES 4
#endif
// The longest Translate / RotateY chain (instances in a row, an outer chain -- a BVH's -- and an
// inner one -- a leaf's inside that BVH -- counted together; round 6: was 4).  reconstruct keeps
// the first 4 in registers and re-walks deeper ones.
#define GS_MAX_CHAIN 16
// Batch rounds (adaptive settings): whole-batch items only for batches up to this size
#ifndef GS_ROUND_WHOLE_MAX_BATCH
#define GS_ROUND_WHOLE_MAX_BATCH 256
#endif
// A split round's per-sample colours: entry a's sample j at j * n + a (sample-major: the
// combine's lanes read one contiguous run per sample), or at a * batch + j (pixel-major: a
// wave's 1-sample items write one contiguous run).  MI355X A2 (round 6): equal render time;
// fabric writes 20.1 vs 15.0 GB a frame, combine 4.2 vs 5.7 ms a frame (5.7 -> 6.2 ms with the
// pixels' samples staged through LDS); profiles/r06/ab_A2_round_items.txt
#ifndef GS_ROUND_PIXEL_MAJOR
#define GS_ROUND_PIXEL_MAJOR 0
#endif
#define GS_NESTED_STACK 32  // max depth of a BVH under a Translate/RotateY chain (a validation bound; the walk is stackless)
// Kernel feature flags (template argument): scenes without them compile the code out.
#define GS_FEAT_MEDIA 1   // ConstantMedium leaves (RNG draws inside traversal)
#define GS_FEAT_NESTED 2  // BVHs under Translate/RotateY (a second-level threaded walk)
#define GS_FEAT_LEAFRUN 4 // sphere leaves come in adjacent pairs: leaf passes test runs of them
#define GS_FEAT_LDSTREE 8 // every record of the threaded tree is in the LDS mirror: no global path
                          // (instantiated without media / nested BVHs only; C3 +1%, C5 +2.5%)
#define GS_FEAT_MIXED 16  // three or more of {sky, Lambertian, metal, dielectric, isotropic}:
                          // staged shading (shade), else one branch per case (shade_split);
                          // media / nested-BVH scenes always stage.  MI355X: C4 +2.2%, C5 +1.6%
                          // staged, C3 (Lambertian + light) -2.8% staged
#define GS_FEAT_VISITS 32 // count tests per threaded record (the placement pilot, run_pilot)
#define GS_FEAT_SPHLEAF 64 // every top-level leaf is a stationary sphere (no media / nested BVHs):
                           // leaf passes without the other kinds' code or the kind test
#ifndef GS_ROOT_RCP
#define GS_ROOT_RCP 1  // sphere roots divided through a refined reciprocal of a (sphere_root_take_ra; A/B: 0)
#endif
#define GS_FEAT_GENERAL 512 // compositions beyond the reference scenes' (round 6): Translate / RotateY chains
                            // deeper than 4, chains inside a BVH under a chain (two-chain hit records), a BVH
                            // as a ConstantMedium boundary, a medium as a medium's boundary.  One catch-all
                            // instantiation (with media, nested BVHs, leaf runs, staged shading); the other
                            // kernels keep the 4-deep single-chain hit record
#define GS_FEAT_PLAIN 256  // staged shading of sphere-only trees whose materials are all solid / two-solid
                           // checker Lambertians, metals and dielectrics with no uv: the hit record of a
                           // stationary sphere only, no texture, light or isotropic code (round 6; C4)
#define GS_FEAT_FIXED 128  // a fixed-spp launch in sample chunks (KParams.chunk != 0, no batch rounds,
                           // max_depth > 0): the adaptive loop's batch ends, stop test, Σlum / Σlum²
                           // and the rounds' per-sample colours are compiled out (round 6)
#define GS_FEAT_RSPLIT 1024  // with GS_FEAT_FIXED: a batch round of split items (KParams.per_sample,
                             // chunk != 0, max_depth > 0) -- the fixed kernel's sample loop, its items
                             // taken from the round's active list and each sample's colour written for
                             // the combine; no stop test, Σlum or batch end in the kernel (round 6)
#ifndef GS_NODE_STEPS
#define GS_NODE_STEPS 8  // node steps per unrolled node pass (the render kernel, below)
#endif
// A wave's issue priority raised (s_setprio level, back to 0 after) while it runs a node pass --
// a chain of dependent LDS reads and box tests, latency-bound per wave -- and, in kernels whose
// leaves are not all stationary spheres and whose leaf passes are not C5's mix (staged shading
// without media or nested BVHs), a leaf pass.  Round 6, MI355X (Msamples/s; none / node
// 1 / node 1 + leaf 1 / node 2 + leaf 1 / node 3): C4 8 773 / 8 971 / 8 886 / 8 911 / 8 962, C3
// 13 969 / 13 992 / 14 204 / 14 179 / 14 011, C2 38 267 / 38 279 / 38 385 / 38 365 / 38 450, C1
// 21 346 / 21 123 / 21 547 / 21 475 / 21 507; none / node 1 / node 1 + leaf 1: C5 7 129 / 7 164 /
// 7 057, final_scene 2 750 / 2 772 / 2 807, cornell_smoke 9 702 / 9 700 / 9 770, A2 11 074 / - /
// 11 333 (profiles/r06/ab_wave_priority.txt).  (FEAT: the kernel's template argument where the
// macros are used.)
#ifndef GS_PRIO_NODE
#define GS_PRIO_NODE 1
#endif
#ifndef GS_PRIO_LEAF
#define GS_PRIO_LEAF                                 \
    ((FEAT & GS_FEAT_SPHLEAF) == 0 &&                \
             ((FEAT & GS_FEAT_MIXED) == 0 || (FEAT & (GS_FEAT_MEDIA | GS_FEAT_NESTED)) != 0) \
         ? 1                                         \
         : 0)
#endif
#ifndef GS_PRIO_SHADE
#define GS_PRIO_SHADE 0
#endif
#define GS_PRIO_SET(lvl) do { if (lvl) __builtin_amdgcn_s_setprio(lvl); } while (0)
#define GS_PRIO_CLR(on) do { if (on) __builtin_amdgcn_s_setprio(0); } while (0)
__host__ __device__ constexpr int unroll_steps(int feat) { return GS_NODE_STEPS; }
// The pilot's instantiation: every code path (any scene), plus the counts.
#define GS_FEAT_PILOT (GS_FEAT_MEDIA | GS_FEAT_NESTED | GS_FEAT_LEAFRUN | GS_FEAT_MIXED | GS_FEAT_VISITS)
#define GS_FEAT_GENERAL_KERNEL (GS_FEAT_GENERAL | GS_FEAT_MEDIA | GS_FEAT_NESTED | GS_FEAT_LEAFRUN | GS_FEAT_MIXED)

// ---------------------------------------------------------------- device layout
// Internal layouts (may differ from the ABI records; converted at upload).
// Material record with the common texture cases folded in (64 B, one line): a
// Lambertian/DiffuseLight over a SolidColorTexture, or over a CheckeredTexture of two
// solids (the bouncing_spheres ground), reads no texture record at shading time.
enum {
    DM_LAMB_SOLID = 1,    // a = albedo
    DM_LAMB_CHECKER = 2,  // a = even, b = odd, param = scale_inv   (texture.rs:58-70)
    DM_LAMB_TEX = 3,      // generic texture tree: `texture`
    DM_METAL = 4,         // a = albedo, param = fuzz
    DM_DIELECTRIC = 5,    // param = refraction index
    DM_LIGHT_SOLID = 6,   // a = emitted colour
    DM_LIGHT_TEX = 7,     // `texture`
    DM_ISO_SOLID = 8,     // Isotropic over a solid: a = albedo  (material.rs:185-196)
    DM_ISO_TEX = 9        // Isotropic over `texture`
};
// ISA census build only (-DGS_ISA_MARKS, tools/isa_census.py): assembler comments that
// delimit the node pass, its f64 fallback and the leaf pass in the generated code.
#ifdef GS_ISA_MARKS
#define GS_MARK(s) asm volatile(";; GS_MARK " s)
#else
#define GS_MARK(s) do { } while (0)
#endif

struct alignas(16) DMaterial {
    uint32_t kind, texture, needs_uv, pad;
    double a[3];
    double param;
    double b[3];
    double pad2;
};

enum { C_RAYS = 0, C_NODES, C_SPH, C_MSPH, C_QUAD, C_TRI, C_INST, C_LIST, C_HITS, C_IMG, C_HDRI, C_PATHS, C_PIX, C_MED, C_NOISE, C_N };
#ifdef GS_CERT_CHECK
#define GS_CNT_SLOTS (C_N + 1)  // + slot 15: nested certified-decision mismatches
#else
#define GS_CNT_SLOTS C_N
#endif

struct DevScene {
    // BVHs under Translate/RotateY chains (GS_FEAT_NESTED): their records are threaded into
    // the node and leaf arrays with the top-level tree's; nroots[k] is the link of tree k's
    // root record (an instance whose chain ends in tree k has the child GS_REF_NODE | k).
    const uint32_t* nroots;
    const DSphere* spheres;
    const uint32_t* sphere_mat;
    const gs_msphere* mspheres;
    const gs_quad* quads;
    const gs_triangle* tris;
    const gs_list* lists;       // (a Quad::cube list: {cube index, GS_CUBE_FLAG | first quad}, cube_test)
    const uint32_t* list_refs;
    const double* cubes;        // GS_CUBE_DOUBLES per Quad::cube list (cube_test)
    const gs_instance* inst;
    const gs_medium* media;
    const uint8_t* noise_perm;  // 256 B, Perlin::default()'s table (NoiseTexture)
    const DMaterial* mats;
    const gs_texture* texs;
    const gs_image* images;
    const uint8_t* texels;
    const float* hdri;
    const uint32_t* hdri_rgbe;  // non-null when every texel round-trips through RGBE8
    gs_background bg;
    uint32_t root;
    // the threaded records (GS_FEAT_GENERAL: a BVH as a medium boundary is walked from global
    // memory by tree_test; the kernels' own walks read them through KArgs and the LDS mirror)
    const TNode* tnodes;
    const TBox* tboxes;
    const TLeaf* tleaves;
};

// Cold launch parameters: written to device memory per launch and read through a
// pointer at their (conditional) use sites, so they are not hoisted into SGPRs for
// the whole kernel (a by-value struct of this size spilled SGPRs into VGPR lanes,
// costing 16 v_readlane per traversal step).
struct KParams {
    DevScene sc;
    gs_camera cam;
    gs_sample_settings ss;
    uint64_t seed;
    int32_t rank, world_size, tile_w, tile_h, tiles_x, pad;
    uint32_t capacity;  // packed pixel slots of this rank
    // Sample chunking (single-batch settings only): work item q = (packed pixel q / cpp,
    // samples [(q % cpp) * chunk, +chunk)); each item leaves its Σrgb in `partial` and
    // gs_combine_kernel sums a pixel's chunks in chunk order.  chunk == 0: one item per
    // pixel running the reference's batch loop (camera.rs:135-165) to completion.
    // `partial` is chunk-major (round 5): chunk ck of coarse pixel k at ck * fine_px + k, of
    // fine pixel k at fine_base + ck * (capacity - fine_px) + k - fine_px, so the combine's
    // lanes (consecutive pixels) read consecutive sums.
    uint32_t chunk, cpp, n_items;
    // Guided tail: the packed pixels from fine_px on (the rank's last tiles in queue order)
    // run in smaller chunks (fine_chunk samples, fine_cpp per pixel), their items (and
    // sums) from fine_base = fine_px * cpp on, so the frame's last items are short (fine_px =
    // capacity: no fine region).
    uint32_t fine_px, fine_base, fine_chunk, fine_cpp;
    uint32_t claim;  // work items a wave claims per queue atomic (its private reserve)
#ifndef GS_CLAIM_DIV
// claims per wave's share of the items (MI355X C1, 25 4-sample chunks per pixel: 8 -> 18 035-
// 18 079, 4 -> 20 335, 2 -> 20 273 Msamples/s; C2, C4, A1, A2 within noise; the coarse
// claims' cap of 32 binds for large frames either way: profiles/r05/ab_claim_div.txt)
#define GS_CLAIM_DIV 4
#endif
#ifndef GS_CLAIM_FINE
// the claim's cap for items of a few samples: one queue counter serialises the claims (MI355X
// C1, 1-2 sample items: cap 32 -> 6786, 128 -> 12397, 512 -> 12559; perlin 3169, 3221, 2670)
#define GS_CLAIM_FINE 128
#endif
    uint32_t claim_fine;  // the same once the wave's claims reach the fine region
    // multiply-shift forms of the launch's fixed divisors (devmath.hpp UDiv): chunks per
    // pixel, tile pixels, 8x8 blocks per tile row, tile width, tiles per row, image width
    UDiv u_cpp, u_tpx, u_bpr, u_tw, u_tx, u_w, u_fcpp;
    const int32_t* order;  // position -> tile (gs_partition.d_tile_order), or null: tile = position
    double* partial;
    float* out;     // linear colour per packed pixel (nullable when out8 is set)
    uint8_t* out8;  // write_color bytes of the f64 colour per packed pixel (nullable)
    // 1: out / out8 are the W x H frame itself (image pixel j * W + i), padding slots are not
    // written -- the one-device frame context, which then needs no unpack (round 5)
    uint32_t direct;
    uint32_t zero_counters;  // 1: gs_params_kernel zeroes `counters` first (the frame context's own buffer)
    unsigned long long* counters;
    uint32_t* queue;
    uint32_t* item_visits;  // diagnostic: node visits per packed pixel (nullable)
    // GS_FEAT_VISITS launches (the placement pilot): tests per node record position, then
    // per leaf record position from visit_leaf_base
    uint32_t* visits;
    uint32_t visit_leaf_base, pad1;
    // Adaptive settings in batch rounds (rounds = 1; DESIGN.md §3.2 "Adaptive sampling in
    // batch rounds"): launch (round, segment) renders batch `round` of the active packed
    // pixels active[seg_base, seg_base + seg_n).  gs_round_params_kernel sets the per-round
    // fields from the device-side counts and picks one of two item forms:
    //  * whole (many pixels active): item = one pixel's whole batch, run in one lane from the
    //    pixel's running sums (pstate) exactly as the per-lane loop runs it, then the stop test
    //    (camera.rs:149-164) in the lane, which writes the colour or the sums and appends the
    //    pixel to the next round's list;
    //  * split (per_sample = 1, few pixels left): item q = (entry q / cpp, samples
    //    [(q % cpp) * chunk, +chunk) of the batch), every sample's colour to partial[(j *
    //    seg_n + entry) * 3] (sample-major: j = the sample's index in the batch); then
    //    gs_round_combine_kernel folds each pixel's batch into its sums in sample order
    //    (camera.rs:138-147) and takes the stop test.
    uint32_t per_sample, round_base, seg_base, seg_n;
    uint32_t waves, lanes, rounds, round;
    const uint32_t* active;    // this round's active packed pixels
    uint32_t* next_active;     // the next round's, appended by the combine
    uint32_t* active_buf[2];   // the two lists (rounds alternate)
    uint32_t* round_counts;    // [rounds + 1]: active pixels per round
    unsigned long long* rpp_hint;  // [2]: rays, paths of the slot's last split rounds (item sizes; kept across launches)
    double* pstate;            // per packed pixel: the running Σr, Σg, Σb, Σlum, Σlum² (camera.rs:131-146)
    // GS_FEAT_NESTED: per lane (block * GS_BLOCK + thread), the top-level ray while the lane
    // walks a BVH under an instance chain: o, d (6 doubles), the return link (u32), and (the
    // general kernel) a hit's outer chain -- slot k of lane g at [k * grid lanes + g]
    double* nest_save;
};

// Hot kernel arguments: what the traversal loop reads every step.
struct KArgs {
    const TNode* tnodes;   // the threaded top-level tree: node records (f32 box, links)
    const TLeaf* tleaves;  // its leaf records
    const TBox* tboxes;    // the f64 box of each node record (undecided / non-cert rays)
    const TQuad* tquads;   // the quads' traversal records (gs_quad order)
    const KParams* P;
    uint32_t root;
    int32_t shade_batch;
    int32_t leaf_batch;  // >= 1: tracing lanes at a leaf before a wave runs a leaf pass
    int32_t node_steps;  // node steps per node pass, 1 .. GS_NODE_STEPS (per scene, see gs_set_node_steps)
    int32_t cam_batch;   // >= 1: lanes waiting for a camera ray before a wave generates them (gs_set_camera_batch)
    int32_t cert_boxes;  // every node coordinate |x| <= 1e15: cert rays may take box_cert
    uint32_t lds_nodes;  // node records [0, lds_nodes) are mirrored in each block's LDS,
    uint32_t lds_leaves; // then leaf records [0, lds_leaves)
    uint32_t lds_quads;  // then quad records [0, lds_quads)
    uint32_t lds_cubes;  // then the Quad::cube records [0, lds_cubes) (cube_test)
    const double* cubes; // (the mirror's source)
    uint32_t lane_nd;    // f64 lane-state fields in LDS: lane_nd(chunked) + nest_lds
    uint32_t nest_lds;   // of which the nested walk's save slots (0: in KParams::nest_save)
};

// S_CAM: the lane's next sample needs its camera ray (set by the refill for a new item and
// by the shade pass for a finished sample; one advance() at the loop head serves both).
enum { S_NEED = 0, S_TRACE = 1, S_SHADE = 2, S_DONE = 3, S_CAM = 4 };

// DevScene::root in the two-child records' terms: a BVH node is its bare index (< 2^26),
// leaves keep their ABI tag (kind >= 2 in the top 4 bits), "none" is all ones.  (The
// kernels start at KArgs::root, the threaded tree's first link; this form is kept for the
// scene record only.)
#define DREF_NONE 0xFFFFFFFFu
#define DREF_LEAF (1u << GS_REF_SHIFT)
__host__ __device__ inline uint32_t device_ref(uint32_t abi_ref) {
    if (abi_ref == GS_REF_NONE) return DREF_NONE;
    if ((abi_ref >> GS_REF_SHIFT) == GS_REF_NODE) return abi_ref & GS_REF_MASK;
    return abi_ref;
}

// Threaded top-level tree.
// BVHNode::hit's left-first recursion (BVH.rs:69-90) visits the tree in pre-order, and a
// box miss skips exactly the node's subtree.  So the top-level tree is stored as its
// pre-order sequence of records — one per node AND one per leaf occurrence — where a node
// record holds its box, a hit link (the next record: its left child) and a miss link (the
// record after its subtree), and a leaf record holds the primitive's ABI ref, a stationary
// sphere's centre/radius inline, and its next link.  The walk is then `cur = hit ? hit_link
// : miss_link` with no stack: the same records tested in the same order with the same
// closest t, minus every push, pop and LDS stack slot.  Links are record indices, a leaf's
// tagged with THR_LEAF; THR_END ends the walk.
#define THR_END 0x7FFFFFFFu
#define THR_LEAF 0x80000000u
// The last links of a BVH under an instance chain (GS_FEAT_NESTED): "back to the top-level
// ray" -- a leaf-tagged value no leaf index reaches (< 2^26), so a lane there waits for a
// leaf pass like a lane at a leaf.
#define THR_RET 0xFFFFFFFFu

// Node and leaf records live in two arrays (32-B TNode, 48-B TLeaf: geometry.hpp); a link
// is a node's byte offset (index << 5: the address arithmetic of a node step is then
// none in LDS and one SGPR-base add in global memory), THR_LEAF | a leaf index, or
// THR_END.  Each block mirrors the most-tested
// prefix of both arrays in LDS.  Address-space-qualified pointers keep the mirror reads
// ds_read instructions: a select between an LDS and a global pointer would compile to
// flat loads, which measured 34% slower on the whole kernel.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) const u32x2 lds_u32x2;
__device__ __forceinline__ double lo_hi(unsigned int lo, unsigned int hi) { return __hiloint2double((int)hi, (int)lo); }

// A node record (2 x 16 B) at byte offset `off`: a = (mnx, mny, mxx, mxy), b = (mnz, mxz,
// hit, miss).  (Offsets are u32: fewer than 2^26 records; leaf offsets i * 48 < 2^32.)
// (Bank-swizzled node and quad records were measured and dropped in round 3: C4 -1.4%,
// C5 -1.3%)
__host__ __device__ constexpr uint32_t node_link(uint32_t pos) { return pos << 5; }
__device__ __forceinline__ uint32_t node_half_b(uint32_t off) { return off + 16u; }
__device__ __forceinline__ uint32_t node_global(uint32_t off) { return off; }
template <bool LDS_ONLY>
__device__ __forceinline__ void load_tnode(const uint8_t* s_nodes, const TNode* g, uint32_t off, uint32_t lds_bytes,
                                           u32x4& a, u32x4& b) {
    if (LDS_ONLY || off < lds_bytes) {
        // The kernel has no static LDS (checked at launch), so the node mirror's first byte
        // is LDS address 0 and `off` is the record's LDS address (no address arithmetic).
        a = *(lds_u32x4*)(uintptr_t)off;
        b = *(lds_u32x4*)(uintptr_t)node_half_b(off);
    } else {
        const u32x4* q = reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(g) + node_global(off));
        a = q[0];
        b = q[1];
    }
}
// The same, for the node steps of a pass: when no active lane's record lies outside the
// mirror (the common case once the mirror holds the most-tested records) the wave takes
// a scalar branch straight to the LDS reads, with no exec-mask split and no wait on
// global loads; otherwise each lane reads its own record's memory.
template <bool LDS_ONLY>
__device__ __forceinline__ void load_tnode_w(const uint8_t* s_nodes, const TNode* g, uint32_t off, uint32_t lds_bytes,
                                             u32x4& a, u32x4& b) {
    if (LDS_ONLY || __builtin_expect(__builtin_amdgcn_ballot_w64(off >= lds_bytes) == 0, 1)) {
        a = *(lds_u32x4*)(uintptr_t)off;
        b = *(lds_u32x4*)(uintptr_t)node_half_b(off);
    } else {
        load_tnode<false>(s_nodes, g, off, lds_bytes, a, b);
    }
}
// 1/d for the f64 slab test on the rare paths.  The asm barrier keeps the compiler from
// hoisting these divisions out of the traversal loop (d is loop-invariant) into six
// registers live across the whole loop: recomputed where needed, they cost nothing in
// the common path.
__device__ __forceinline__ d3 inv_of(d3 d) {
    asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z));
    return mk(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
}
__device__ __forceinline__ d3 inv_cert(d3 d) {
    asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z));  // (as inv_of: not hoisted)
    return mk(rcp_cert(d.x), rcp_cert(d.y), rcp_cert(d.z));
}
// Chunk sums and per-sample colours (written once, read by the combine kernel).  (Non-temporal
// stores measured neutral, C4 +0.2%, final_scene +0.7%, and wrote as many fabric bytes: gfx950
// stores leave L2 whatever their flavour, MI355X_MICROARCH.md; profiles/r06/ab_nt_partial.txt.)
__device__ __forceinline__ void st_partial(double* o, double r, double g, double b) {
    o[0] = r;
    o[1] = g;
    o[2] = b;
}
// A leaf record: the sphere's centre and radius squared, its next link and its ABI ref.
template <bool LDS_ONLY>
__device__ __forceinline__ void load_tleaf(const uint8_t* s_leaves, const TLeaf* g, uint32_t i, uint32_t lds_l,
                                           double& cx, double& cy, double& cz, double& rr, uint32_t& next,
                                           uint32_t& ref) {
    u32x4 a, b;
    u32x2 d;
    // (as load_tnode_w: one scalar branch when every active lane's record is mirrored)
    if (LDS_ONLY || __builtin_expect(__builtin_amdgcn_ballot_w64(i >= lds_l) == 0, 1)) {
        const uint8_t* p = s_leaves + i * 48u;
        a = ((lds_u32x4*)p)[0];
        b = ((lds_u32x4*)p)[1];
        d = *(lds_u32x2*)(p + 32);
    } else if (i < lds_l) {
        const uint8_t* p = s_leaves + i * 48u;
        a = ((lds_u32x4*)p)[0];
        b = ((lds_u32x4*)p)[1];
        d = *(lds_u32x2*)(p + 32);
    } else {
        const char* p = reinterpret_cast<const char*>(g) + i * 48u;
        a = reinterpret_cast<const u32x4*>(p)[0];
        b = reinterpret_cast<const u32x4*>(p)[1];
        d = *reinterpret_cast<const u32x2*>(p + 32);
    }
    cx = lo_hi(a.x, a.y);
    cy = lo_hi(a.z, a.w);
    cz = lo_hi(b.x, b.y);
    rr = lo_hi(b.z, b.w);
    next = d.x;
    ref = d.y;
}

// Quad records for traversal (TQuad): [0, n_lds) from the block's LDS mirror, the rest
// from global memory; 16 B at a time, so a quad whose plane misses reads 32 B, not 128.
struct QuadSrc {
    const uint8_t* lds;
    const TQuad* g;
    uint32_t n_lds;
    // the Quad::cube records mirrored in LDS: [0, n_lcubes) at lcubes (cube_test)
    const uint8_t* lcubes;
    uint32_t n_lcubes;
};

// Scene-record loads of the leaf tests, field by field through a pointer of an explicit
// address space: global (vector loads) or, with UNI — every active lane tests the same
// leaf, a wave-uniform ref — constant, which compiles to scalar loads (the scalar cache:
// no vector-memory instruction, no per-lane address, uniform branches after them).  The
// scene's pointers are generic and load through flat instructions otherwise (which also
// count against lgkmcnt); a whole-struct copy from constant memory is rewritten by the
// optimiser into flat loads again, hence the field-wise copies.
#ifdef __HIP_DEVICE_COMPILE__
#define GS_SCENE_AS(UNI) __attribute__((address_space((UNI) ? 4 : 1)))
#else
#define GS_SCENE_AS(UNI)
#endif
template <bool UNI, class T>
__device__ __forceinline__ const GS_SCENE_AS(UNI) T* sp(const T* p) {
    return (const GS_SCENE_AS(UNI) T*)p;
}
template <bool UNI>
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
    return *sp<UNI>(p);
}
template <bool UNI>
__device__ __forceinline__ gs_instance ld_inst(const gs_instance* p) {
    const auto q = sp<UNI>(p);
    gs_instance v;
    v.kind = q->kind;
    v.child = q->child;
    v.p[0] = q->p[0];
    v.p[1] = q->p[1];
    v.p[2] = q->p[2];
    return v;
}
template <bool UNI>
__device__ __forceinline__ gs_list ld_list(const gs_list* p) {
    const auto q = sp<UNI>(p);
    gs_list v;
    v.first = q->first;
    v.count = q->count;
    return v;
}
template <bool UNI>
__device__ __forceinline__ gs_medium ld_medium(const gs_medium* p) {
    const auto q = sp<UNI>(p);
    gs_medium v;
    v.boundary = q->boundary;
    v.material = q->material;
    v.density_neg_inv = q->density_neg_inv;
    return v;
}
template <bool UNI>
__device__ __forceinline__ u32x4 quad_part(const QuadSrc& qs, uint32_t i, uint32_t k) {
    if (!UNI && i < qs.n_lds) return *(lds_u32x4*)(qs.lds + i * (uint32_t)sizeof(TQuad) + (k << 4));
    return sp<UNI>(reinterpret_cast<const u32x4*>(qs.g + i))[k];
}
// The aligned form's tag (aligned_tquad, host: the cube records' derivation): a
// signalling-NaN first word carrying the axis code 2 a + o.  (Single quads in the aligned
// form, with per-lane selects or compile-time copies per axis code, were measured and
// dropped in round 4, profiles/r04/ab_aligned_quads.txt.)
#define GS_AQ_TAG 0xFFF4A5C0u
template <int CODE>
__device__ __forceinline__ double d3_c(const d3& v, int which) {  // which: 0 = a, 1 = iu, 2 = iv
    constexpr int A = CODE >> 1, O = CODE & 1;
    const int k = which == 0 ? A : (which == 1 ? (A + 1 + O) % 3 : (A + 2 - O) % 3);
    return k == 0 ? v.x : (k == 1 ? v.y : v.z);
}
template <bool UNI>
__device__ __forceinline__ bool quad_test(const QuadSrc& qs, uint32_t i, const Ray& ray, double tmin, double tmax,
                                          double& t_out) {
    const u32x4 a = quad_part<UNI>(qs, i, 0);
    const u32x4 b = quad_part<UNI>(qs, i, 1);
    return quad_accept_plane(
        mk(lo_hi(a.x, a.y), lo_hi(a.z, a.w), lo_hi(b.x, b.y)), lo_hi(b.z, b.w),
        [&](d3& Q, d3& U, d3& V, d3& W) {
            const u32x4 c = quad_part<UNI>(qs, i, 2), e = quad_part<UNI>(qs, i, 3), f = quad_part<UNI>(qs, i, 4);
            const u32x4 g = quad_part<UNI>(qs, i, 5), h = quad_part<UNI>(qs, i, 6), m = quad_part<UNI>(qs, i, 7);
            Q = mk(lo_hi(c.x, c.y), lo_hi(c.z, c.w), lo_hi(e.x, e.y));
            U = mk(lo_hi(e.z, e.w), lo_hi(f.x, f.y), lo_hi(f.z, f.w));
            V = mk(lo_hi(g.x, g.y), lo_hi(g.z, g.w), lo_hi(h.x, h.y));
            W = mk(lo_hi(h.z, h.w), lo_hi(m.x, m.y), lo_hi(m.z, m.w));
        },
        ray, tmin, tmax, t_out);
}

__device__ __forceinline__ bool cur_next_is_leaf(uint32_t link) { return link > THR_END; }

// Outcome of testing one non-node child against the ray.
struct LeafHit {
    bool hit;
    double t;
    uint32_t ref, inst;
    uint32_t enter;  // GS_FEAT_NESTED: the chain ended in BVH tree `enter - 1` (0: it did not)
};

// One primitive ref against `ray` (already in the primitive's space); accepts into
// `res` ("last accepted wins", as BVH.rs:73-80 and hittable.rs:75-83 compose).
template <bool UNI>
__device__ __forceinline__ void prim_test(const DevScene& sc, const QuadSrc& qs, uint32_t ref, const Ray& ray,
                                          double tmin, double closest, uint32_t inst_ref, LeafHit& res,
                                          unsigned long long* cnt) {
    const uint32_t kind = ref >> GS_REF_SHIFT, idx = ref & GS_REF_MASK;
    double t;
    bool ok = false;
    if (kind == GS_REF_SPHERE) {
        atomicAdd(&cnt[C_SPH], 1ull);
        const auto s = sp<UNI>(sc.spheres + idx);
        ok = sphere_accept(mk(s->cx, s->cy, s->cz), s->r, ray, len2(ray.d), tmin, closest, t);
    } else if (kind == GS_REF_MSPHERE) {
        atomicAdd(&cnt[C_MSPH], 1ull);
        const auto s = sp<UNI>(sc.mspheres + idx);
        const d3 c0 = mk(s->center_start[0], s->center_start[1], s->center_start[2]);
        const d3 cp = mk(s->center_path[0], s->center_path[1], s->center_path[2]);
        d3 c = add(c0, muls(cp, ray.time));
        ok = sphere_accept(c, s->radius, ray, len2(ray.d), tmin, closest, t);
    } else if (kind == GS_REF_QUAD) {
        atomicAdd(&cnt[C_QUAD], 1ull);
        ok = quad_test<UNI>(qs, idx, ray, tmin, closest, t);
    } else if (kind == GS_REF_TRIANGLE) {
        atomicAdd(&cnt[C_TRI], 1ull);
        double u, v;
        const auto q = sp<UNI>(sc.tris + idx);
        gs_triangle tr;
        for (int k = 0; k < 3; k++) {
            tr.a[k] = q->a[k];
            tr.b[k] = q->b[k];
            tr.c[k] = q->c[k];
        }
        ok = tri_hit(tr, ray, t, u, v);
    }
    if (ok) {
        res.hit = true;
        res.t = t;
        res.ref = ref;
        res.inst = inst_ref;
    }
}

// Translate / RotateY chain (hittable.rs:107-113, :179-193): the ray in the innermost
// child's space; returns that child's ref.
template <bool UNI>
__device__ __forceinline__ uint32_t walk_chain(const DevScene& sc, uint32_t cur, Ray& r, unsigned long long* cnt) {
#pragma unroll 1
    for (int k = 0; k < GS_MAX_CHAIN && (cur >> GS_REF_SHIFT) == GS_REF_INSTANCE; k++) {
        const gs_instance in = ld_inst<UNI>(sc.inst + (cur & GS_REF_MASK));
        atomicAdd(&cnt[C_INST], 1ull);
        inst_forward(in, r);
        cur = in.child;
    }
    return cur;
}

// The instance tests of walking a chain again (counted, nothing computed).
template <bool UNI>
__device__ __forceinline__ void chain_count(const DevScene& sc, uint32_t cur, unsigned long long* cnt) {
#pragma unroll 1
    for (int k = 0; k < GS_MAX_CHAIN && (cur >> GS_REF_SHIFT) == GS_REF_INSTANCE; k++) {
        atomicAdd(&cnt[C_INST], 1ull);
        cur = ld_u32<UNI>(&sc.inst[cur & GS_REF_MASK].child);
    }
}

// A Quad::cube list (quad.rs:54-80: six quads in a fixed order, all axis-aligned, added one
// after the other) as straight-line code: face k's plane axis and in-plane axes are
// compile-time constants (cube_code: the aligned form's 2 a + o), so each face is Quad::hit
// in the reduced form aquad_accept states -- the same t, alpha and beta bit for bit -- with
// no selects and no loop, in the list's order with its shrinking closest (hittable.rs:
// 71-86).  Every face value is one of twelve numbers of the box: its corners min = (x0, y0,
// z0) and max = (x1, y1, z1), the edges dx, dy, dz and the three w magnitudes (w_xy of the
// z faces, w_zy of the x faces, w_xz of the y faces), with a sign: the 96-B record
// [x0 y0 z0 x1 y1 z1 dx dy dz w_xy w_zy w_xz] (a negation is exact and free, an f64
// operand modifier).  The host (cube_record) builds a cube only when all six faces' aligned
// records equal what this table derives; the other lists keep the loop.
#define GS_CUBE_FLAG 0x80000000u
#define GS_CUBE_DOUBLES 12
__host__ __device__ constexpr int cube_code(int k) { return k == 0 || k == 2 ? 4 : (k == 1 || k == 3 ? 1 : 3); }
// face k's D', Q_iu, Q_iv, U_iu, V_iv, W' as (record index, sign): quad.rs:73-78 in order
__host__ __device__ constexpr int cube_src(int k, int f) {
    constexpr int t[6][6] = {{5, 0, 1, 6, 7, 9},    {3, 5, 1, -8, 7, -10}, {2, 3, 1, -6, 7, -9},
                             {0, 2, 1, 8, 7, 10},   {4, 0, 5, 6, -8, -11}, {1, 0, 2, 6, 8, 11}};
    return t[k][f];
}
// (the record is read up front: faces reading their values lazily measured -0.3 to -2.8%)
struct CubeRegs {
    double c[GS_CUBE_DOUBLES];
    template <int J>
    __device__ __forceinline__ double get() const { return c[J]; }
};
template <bool UNI>
__device__ __forceinline__ u32x4 cube_part(const QuadSrc& qs, const double* g, uint32_t cube, uint32_t k, bool lds) {
    if (!UNI && lds) return *(lds_u32x4*)(qs.lcubes + cube * (uint32_t)(GS_CUBE_DOUBLES * 8) + (k << 4));
    return sp<UNI>(reinterpret_cast<const u32x4*>(g + (size_t)cube * GS_CUBE_DOUBLES))[k];
}
template <int K, int F, class Src>
__device__ __forceinline__ double cube_val(const Src& c) {
    constexpr int v = cube_src(K, F);
    if constexpr (v < 0) return -c.template get<-v>();
    else return c.template get<v>();
}
template <int K, class Src>
__device__ __forceinline__ void cube_face(const Src& c, uint32_t q0, const Ray& r, double tmin, uint32_t inst_ref,
                                          LeafHit& res) {
    constexpr int C = cube_code(K);
    const double da = d3_c<C>(r.d, 0);
    if (fabs(da) < 1e-8) return;
    const double t = (cube_val<K, 0>(c) - d3_c<C>(r.o, 0)) / da;
    if (!(tmin <= t && t <= res.t)) return;
    const double pu = (d3_c<C>(r.o, 1) + d3_c<C>(r.d, 1) * t) - cube_val<K, 1>(c);
    const double pv = (d3_c<C>(r.o, 2) + d3_c<C>(r.d, 2) * t) - cube_val<K, 2>(c);
    const double W = cube_val<K, 5>(c);
    const double alpha = W * (pu * cube_val<K, 4>(c));
    const double beta = W * (cube_val<K, 3>(c) * pv);
    if (!(0.0 <= alpha && alpha <= 1.0) || !(0.0 <= beta && beta <= 1.0)) return;
    res.hit = true;
    res.t = t;
    res.ref = GS_MAKE_REF(GS_REF_QUAD, q0 + K);
    res.inst = inst_ref;
}
template <class Src>
__device__ __forceinline__ void cube_faces(const Src& c, uint32_t q0, const Ray& r, double tmin, uint32_t inst_ref,
                                           LeafHit& res) {
    cube_face<0>(c, q0, r, tmin, inst_ref, res);
    cube_face<1>(c, q0, r, tmin, inst_ref, res);
    cube_face<2>(c, q0, r, tmin, inst_ref, res);
    cube_face<3>(c, q0, r, tmin, inst_ref, res);
    cube_face<4>(c, q0, r, tmin, inst_ref, res);
    cube_face<5>(c, q0, r, tmin, inst_ref, res);
}
template <bool UNI>
__device__ __forceinline__ void cube_test(const DevScene& sc, const QuadSrc& qs, uint32_t cube, uint32_t q0,
                                          const Ray& r, double tmin, uint32_t inst_ref, LeafHit& res,
                                          unsigned long long* cnt) {
    atomicAdd(&cnt[C_QUAD], 6ull);
    CubeRegs c;
    // the LDS copy when every lane's cube is mirrored (a wave-uniform choice: a per-lane
    // one ran both kinds of loads under masks, final_scene -2.3%), else global for all
    const bool lds = !UNI && __builtin_amdgcn_ballot_w64(cube >= qs.n_lcubes) == 0;
#pragma unroll
    for (uint32_t k = 0; k < GS_CUBE_DOUBLES / 2; k++) {
        const u32x4 v = cube_part<UNI>(qs, sc.cubes, cube, k, lds);
        c.c[2 * k] = lo_hi(v.x, v.y);
        c.c[2 * k + 1] = lo_hi(v.z, v.w);
    }
    cube_faces(c, q0, r, tmin, inst_ref, res);
}

// A HittableList (hittable.rs:71-86: shrinking closest) or one primitive.
template <bool UNI>
__device__ __forceinline__ void shape_test(const DevScene& sc, const QuadSrc& qs, uint32_t cur, const Ray& r,
                                           double tmin, double closest, uint32_t inst_ref, LeafHit& res,
                                           unsigned long long* cnt) {
    if ((cur >> GS_REF_SHIFT) == GS_REF_LIST) {
        atomicAdd(&cnt[C_LIST], 1ull);
        const gs_list l = ld_list<UNI>(sc.lists + (cur & GS_REF_MASK));
        if (l.count & GS_CUBE_FLAG) {
            cube_test<UNI>(sc, qs, l.first, l.count & ~GS_CUBE_FLAG, r, tmin, inst_ref, res, cnt);
        } else {
#pragma unroll 1
            for (uint32_t k = 0; k < l.count; k++)
                prim_test<UNI>(sc, qs, ld_u32<UNI>(sc.list_refs + l.first + k), r, tmin, res.t, inst_ref, res, cnt);
        }
    } else {
        prim_test<UNI>(sc, qs, cur, r, tmin, closest, inst_ref, res, cnt);
    }
}

// GS_FEAT_GENERAL: the closest hit of `r` over BVH tree `tree` (threaded like the BVHs under
// instances, its last links THR_RET) in [tmin, res.t] -- BVHNode::hit (BVH.rs:69-90) as its
// pre-order walk with the shrinking closest, every node tested with the reference's f64 slab
// test (AABB.rs:58-113) and counted, the leaves' lists and primitives by shape_test.  For a
// BVH as a ConstantMedium boundary: a rare path, read from global memory.
template <bool UNI>
__device__ __forceinline__ void tree_test(const DevScene& sc, const QuadSrc& qs, uint32_t tree, const Ray& r, double tmin,
                                          LeafHit& res, unsigned long long* cnt) {
    uint32_t link = sc.nroots[tree];
    const d3 inv = inv_of(r.d);
#pragma unroll 1
    for (uint32_t guard = 0; link != THR_RET && guard < (1u << 27); guard++) {
        if (link < THR_END) {  // a node record (its byte offset)
            atomicAdd(&cnt[C_NODES], 1ull);
            const TNode& n = sc.tnodes[link >> 5];
            link = box_hit(box64(sc.tboxes[link >> 5]), r.o, inv, tmin, res.t) ? n.hit : n.miss;
        } else {  // a leaf record
            const TLeaf& lf = sc.tleaves[link & ~THR_LEAF];
            shape_test<false>(sc, qs, lf.ref, r, tmin, res.t, GS_REF_NONE, res, cnt);
            link = lf.next;
        }
    }
}

template <bool UNI, int LEVEL>
__device__ __forceinline__ void medium_test(const DevScene& sc, const QuadSrc& qs, uint32_t cur, const Ray& r, double tmin,
                                            double closest, uint32_t inst_ref, uint64_t& rng, LeafHit& res,
                                            unsigned long long* cnt, bool general);
// A medium's boundary in [tmin, DMAX]: a primitive or list; with GS_FEAT_GENERAL also a BVH
// (tree_test) or, one level deep, another medium (its own ConstantMedium::hit, drawing from
// the lane's stream in the reference's order: volume.rs:36-41 calls boundary.hit twice).
template <bool UNI, int LEVEL>
__device__ __forceinline__ void boundary_test(const DevScene& sc, const QuadSrc& qs, uint32_t shape, const Ray& rb,
                                              double tmin, uint64_t& rng, LeafHit& b, unsigned long long* cnt,
                                              bool general) {
    if (general && (shape >> GS_REF_SHIFT) == GS_REF_NODE) {
        tree_test<UNI>(sc, qs, shape & GS_REF_MASK, rb, tmin, b, cnt);
    } else if (LEVEL == 0 && general && (shape >> GS_REF_SHIFT) == GS_REF_MEDIUM) {
        medium_test<false, 1>(sc, qs, shape, rb, tmin, b.t, GS_REF_NONE, rng, b, cnt, true);
    } else {
        shape_test<UNI>(sc, qs, shape, rb, tmin, b.t, GS_REF_NONE, b, cnt);
    }
}

// ConstantMedium::hit (volume.rs:32-63): the boundary hit over Interval::UNIVERSE, again
// from t1 + 0.0001, both clipped to ray_t; then the free-flight distance from the lane's
// RNG stream, drawn here, inside traversal, in the reference's visit order (:48).
// `general` (GS_FEAT_GENERAL kernels): the boundary may be a BVH or a medium (boundary_test).
template <bool UNI, int LEVEL>
__device__ __forceinline__ void medium_test(const DevScene& sc, const QuadSrc& qs, uint32_t cur, const Ray& r, double tmin,
                                            double closest, uint32_t inst_ref, uint64_t& rng, LeafHit& res,
                                            unsigned long long* cnt, bool general) {
    atomicAdd(&cnt[C_MED], 1ull);
    // the boundary now, the density only where it is used (not held through both hits)
    const gs_medium* mp = sc.media + (cur & GS_REF_MASK);
    struct {
        uint32_t boundary;
    } md{ld_u32<UNI>(&mp->boundary)};
    const double DMAX = 1.7976931348623157e308;  // f64::MAX; f64::MIN = -f64::MAX
    // |ray.d| now (the same value volume.rs:55 computes at the end), so the ray itself is
    // not live through the boundary tests: they need only its transform into the
    // boundary's space, which the second boundary.hit call (volume.rs:38-41) would recompute
    // from the same ray bit for bit -- it is reused, and the second walk's instance tests
    // are counted.  (Without it media kernels spill 12-20 B/lane around the cube tests of
    // box boundaries.)
    const double ray_len = sqrt(len2(r.d));
    LeafHit b1;
    b1.hit = false;
    b1.t = DMAX;
    Ray rb = r;
    const uint32_t shape = walk_chain<UNI>(sc, md.boundary, rb, cnt);
    if (general) boundary_test<UNI, LEVEL>(sc, qs, shape, rb, -DMAX, rng, b1, cnt, true);
    else shape_test<UNI>(sc, qs, shape, rb, -DMAX, DMAX, GS_REF_NONE, b1, cnt);
    if (!b1.hit) return;
    chain_count<UNI>(sc, md.boundary, cnt);
    LeafHit b2;
    b2.hit = false;
    b2.t = DMAX;
    if (general) boundary_test<UNI, LEVEL>(sc, qs, shape, rb, b1.t + 0.0001, rng, b2, cnt, true);
    else shape_test<UNI>(sc, qs, shape, rb, b1.t + 0.0001, DMAX, GS_REF_NONE, b2, cnt);
    if (!b2.hit) return;
    double t1 = b1.t, t2 = b2.t;
    if (t1 < tmin) t1 = tmin;
    if (t2 > closest) t2 = closest;
    if (t1 >= t2) return;
    if (t1 < 0.0) t1 = 0.0;
    const double dist_inside_boundary = (t2 - t1) * ray_len;
    const double hit_dist = sp<UNI>(mp)->density_neg_inv * log(wy_f64(rng));
    if (hit_dist > dist_inside_boundary) return;
    res.hit = true;
    res.t = t1 + hit_dist / ray_len;
    res.ref = cur;
    res.inst = inst_ref;
}

// The rarer non-node children (everything but a stationary sphere reached directly
// from a BVH node): moving sphere, quad, triangle, HittableList, ConstantMedium, behind an
// optional Translate/RotateY chain.  `rng`: a medium draws from the lane's stream.  FEAT
// (GS_FEAT_*) is a kernel template argument: scenes without media compile the medium
// test out (it costs the traversal loop 4 VGPRs and spills otherwise).
// A chain that ends in a BVH (GS_FEAT_NESTED: final_scene's box of balls, main.rs:741-755)
// is not walked here: `r` is left in the tree's space and `enter` = tree + 1, and the
// caller walks the tree in the main loop's passes (round 5; see the leaf pass).
template <int FEAT, bool UNI>
__device__ GS_NOINLINE LeafHit leaf_other(const DevScene& sc, const QuadSrc& qs, uint32_t ref, Ray& r, double tmin,
                                           double closest, uint64_t& rng, unsigned long long* cnt) {
    LeafHit res;
    res.hit = false;
    res.t = closest;
    res.ref = GS_REF_NONE;
    res.inst = GS_REF_NONE;
    res.enter = 0;
    const uint32_t inst_ref = (ref >> GS_REF_SHIFT) == GS_REF_INSTANCE ? ref : GS_REF_NONE;
    const uint32_t cur = walk_chain<UNI>(sc, ref, r, cnt);
    if ((FEAT & GS_FEAT_MEDIA) && (cur >> GS_REF_SHIFT) == GS_REF_MEDIUM) {
        medium_test<UNI, 0>(sc, qs, cur, r, tmin, closest, inst_ref, rng, res, cnt, (FEAT & GS_FEAT_GENERAL) != 0);
    } else if ((FEAT & GS_FEAT_NESTED) && (cur >> GS_REF_SHIFT) == GS_REF_NODE) {
        res.enter = (cur & GS_REF_MASK) + 1u;
    } else {
        shape_test<UNI>(sc, qs, cur, r, tmin, closest, inst_ref, res, cnt);
    }
    return res;
}

struct HitRec {
    d3 p, n;
    double u, v;
    uint32_t mat;
    bool front;
};

__device__ __forceinline__ void sphere_uv(d3 p, double& u, double& v) {  // sphere.rs:55-60
    const double PI = 3.14159265358979323846;
    double theta = acos(-p.y);
    double phi = atan2(-p.z, p.x) + PI;
    u = phi / (2.0 * PI);
    v = theta / PI;
}

// Recompute the HitRecord of the accepted primitive at t (the values the reference
// built when it accepted it), then apply the instance back-transforms innermost-first.
// hit_inst: the chain the hit came through (GS_REF_NONE: none); outer: for a hit through a
// chain inside a BVH that is itself under a chain (round 6), that BVH's chain (applied first
// going in, last coming out), else GS_REF_NONE.
// The n-th instance of the concatenated chain (outer's, then hit_inst's).
__device__ __forceinline__ uint32_t chain_at(const DevScene& sc, uint32_t outer, uint32_t inner, int n) {
    uint32_t cur = outer != GS_REF_NONE ? outer : inner;
    bool in_outer = outer != GS_REF_NONE;
#pragma unroll 1
    for (int k = 0; k < 2 * GS_MAX_CHAIN; k++) {
        if ((cur >> GS_REF_SHIFT) != GS_REF_INSTANCE) {  // the outer chain ended: the inner one
            if (!in_outer) break;
            in_outer = false;
            cur = inner;
            k--;
            continue;
        }
        if (n-- == 0) return cur & GS_REF_MASK;
        cur = sc.inst[cur & GS_REF_MASK].child;
    }
    return 0u;
}
template <bool DEEP>  // GS_FEAT_GENERAL kernels: chains longer than 4, two chains
__device__ GS_NOINLINE HitRec reconstruct(const DevScene& sc, Ray r, double t, uint32_t hit_ref,
                                           uint32_t hit_inst, uint32_t outer = GS_REF_NONE) {
    HitRec h;
    uint32_t ch0 = 0, ch1 = 0, ch2 = 0, ch3 = 0;
    int nch = 0;
    bool deep = DEEP && outer != GS_REF_NONE;  // two chains, or one longer than 4: the re-walking path
    if (hit_inst != GS_REF_NONE && !deep) {
        uint32_t cur = hit_inst;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if ((cur >> GS_REF_SHIFT) != GS_REF_INSTANCE) break;
            uint32_t i = cur & GS_REF_MASK;
            if (k == 0) ch0 = i; else if (k == 1) ch1 = i; else if (k == 2) ch2 = i; else ch3 = i;
            nch = k + 1;
            const gs_instance& in = sc.inst[i];
            inst_forward(in, r);
            cur = in.child;
        }
        if (DEEP && (cur >> GS_REF_SHIFT) == GS_REF_INSTANCE) {  // deeper than 4: on through the rest
            deep = true;
#pragma unroll 1
            for (int k = 4; k < GS_MAX_CHAIN && (cur >> GS_REF_SHIFT) == GS_REF_INSTANCE; k++) {
                const gs_instance& in = sc.inst[cur & GS_REF_MASK];
                inst_forward(in, r);
                cur = in.child;
                nch = k + 1;
            }
        }
    } else if (DEEP && deep) {  // the outer chain, then the inner one
        uint32_t cur = outer;
        bool in_outer = true;
#pragma unroll 1
        for (int k = 0; k < 2 * GS_MAX_CHAIN; k++) {
            if ((cur >> GS_REF_SHIFT) != GS_REF_INSTANCE) {
                if (!in_outer || hit_inst == GS_REF_NONE) break;
                in_outer = false;
                cur = hit_inst;
                continue;
            }
            const gs_instance& in = sc.inst[cur & GS_REF_MASK];
            inst_forward(in, r);
            cur = in.child;
            nch++;
        }
    }
    const uint32_t kind = hit_ref >> GS_REF_SHIFT, idx = hit_ref & GS_REF_MASK;
    d3 p, outward;
    double u = 0.0, v = 0.0;
    if (kind == GS_REF_SPHERE || kind == GS_REF_MSPHERE) {
        d3 c;
        double rad;
        if (kind == GS_REF_SPHERE) {
            DSphere s = sc.spheres[idx];
            c = mk(s.cx, s.cy, s.cz);
            rad = s.r;
            h.mat = sc.sphere_mat[idx];
        } else {
            const gs_msphere& s = sc.mspheres[idx];
            c = add(ld3(s.center_start), muls(ld3(s.center_path), r.time));
            rad = s.radius;
            h.mat = s.material;
        }
        p = add(r.o, muls(r.d, t));
        outward = divs(sub(p, c), rad);
        if (sc.mats[h.mat].needs_uv) sphere_uv(outward, u, v);
    } else if (kind == GS_REF_QUAD) {
        const gs_quad& q = sc.quads[idx];
        p = add(r.o, muls(r.d, t));
        d3 planar = sub(p, ld3(q.q));
        u = dot(ld3(q.w), cross(planar, ld3(q.v)));
        v = dot(ld3(q.w), cross(ld3(q.u), planar));
        outward = ld3(q.normal);
        h.mat = q.material;
    } else if (kind == GS_REF_MEDIUM) {  // volume.rs:54-62: ray.at(t), normal (1, 0, 0), u = v = 0
        p = add(r.o, muls(r.d, t));
        outward = mk(1.0, 0.0, 0.0);
        h.mat = sc.media[idx].material;
    } else {  // triangle
        const gs_triangle& tr = sc.tris[idx];
        double tt;
        tri_hit(tr, r, tt, u, v);
        p = add(r.o, muls(r.d, t));
        outward = ld3(tr.normal);
        h.mat = tr.material;
    }
    // HitRecord::new (hittable.rs:26-43)
    h.front = dot(r.d, outward) < 0.0;
    d3 n = h.front ? outward : neg(outward);
    // Innermost instance first (RotateY inside Translate: rotate back, then translate).
    if (!DEEP || !deep) {
        if (nch > 3) inst_backward(sc.inst[ch3], p, n);
        if (nch > 2) inst_backward(sc.inst[ch2], p, n);
        if (nch > 1) inst_backward(sc.inst[ch1], p, n);
        if (nch > 0) inst_backward(sc.inst[ch0], p, n);
    } else {
#pragma unroll 1
        for (int k = nch - 1; k >= 0; k--) inst_backward(sc.inst[chain_at(sc, outer, hit_inst, k)], p, n);
    }
    h.p = p;
    h.n = n;
    h.u = u;
    h.v = v;
    return h;
}

// The same for a hit that can only be a stationary sphere outside any instance (sphere-only
// trees, GS_FEAT_SPHLEAF): reconstruct's sphere branch and HitRecord::new, nothing else; UV
// false when no material needs uv (GS_FEAT_PLAIN).
template <bool UV>
__device__ __forceinline__ HitRec reconstruct_sphere(const DevScene& sc, const Ray& r, double t, uint32_t hit_ref) {
    HitRec h;
    const uint32_t idx = hit_ref & GS_REF_MASK;
    const DSphere s = sc.spheres[idx];
    const d3 c = mk(s.cx, s.cy, s.cz);
    h.mat = sc.sphere_mat[idx];
    const d3 p = add(r.o, muls(r.d, t));
    const d3 outward = divs(sub(p, c), s.r);
    h.u = 0.0;
    h.v = 0.0;
    if (UV && sc.mats[h.mat].needs_uv) sphere_uv(outward, h.u, h.v);
    h.front = dot(r.d, outward) < 0.0;  // hittable.rs:26-43
    h.n = h.front ? outward : neg(outward);
    h.p = p;
    return h;
}

// Texture::value_at (texture.rs:27-95); checkered nesting resolved iteratively.
__device__ GS_NOINLINE d3 texture_value(const DevScene& sc, uint32_t tex, double u, double v, d3 p,
                                         unsigned long long* cnt) {
#pragma unroll 1
    for (int depth = 0; depth < 16; depth++) {
        const gs_texture& t = sc.texs[tex];
        if (t.kind == GS_TEX_SOLID) return ld3(t.color);
        if (t.kind == GS_TEX_CHECKERED) {
            int32_t xi = sat_i32(floor(t.scale_inv * p.x));
            int32_t yi = sat_i32(floor(t.scale_inv * p.y));
            int32_t zi = sat_i32(floor(t.scale_inv * p.z));
            int32_t s = (int32_t)((uint32_t)xi + (uint32_t)yi + (uint32_t)zi);
            tex = (s % 2 == 0) ? t.even : t.odd;
            continue;
        }
        if (t.kind == GS_TEX_NOISE) {  // texture.rs:127-130
            atomicAdd(&cnt[C_NOISE], 1ull);
            const double n = noise_value(sc.noise_perm, t.color[0], p.x, p.y, p.z);
            return mk(n, n, n);
        }
        // GS_TEX_IMAGE
        const gs_image im = sc.images[t.image];
        double uc = u, vc = v;
        if (uc < 0.0) uc = 0.0;
        if (uc > 1.0) uc = 1.0;
        if (vc < 0.0) vc = 0.0;
        if (vc > 1.0) vc = 1.0;
        vc = 1.0 - vc;
        uint64_t i = sat_u64(uc * (double)im.width, 4294967295.0, 4294967295ull);
        uint64_t j = sat_u64(vc * (double)im.height, 4294967295.0, 4294967295ull);
        if (i > im.width - 1) i = im.width - 1;  // reference panics here (u == 1); documented clamp
        if (j > im.height - 1) j = im.height - 1;
        const uint8_t* px = sc.texels + im.offset + (j * (uint64_t)im.width + i) * 3;
        atomicAdd(&cnt[C_IMG], 1ull);
        return muls(mk((double)px[0], (double)px[1], (double)px[2]), 1.0 / 255.0);
    }
    return mk(0.0, 0.0, 0.0);
}

// HDRI::sample's texel (camera.rs:257-270) for an already normalised, rotated direction.
__device__ __forceinline__ d3 hdri_texel(const DevScene& sc, d3 rot, unsigned long long* cnt) {
    const gs_background& bg = sc.bg;
    uint32_t x, y;
    // f32 angles where they certify the texel, else the reference's f64 atan2 / asin
    // (sky_index_f32 / sky_index_f64, geometry.hpp)
    if (!sky_index_f32(rot, bg.width, bg.height, x, y)) sky_index_f64(rot, bg.width, bg.height, x, y);
    const uint64_t k = y * (uint64_t)bg.width + x;
    atomicAdd(&cnt[C_HDRI], 1ull);
    if (sc.hdri_rgbe) {
        // RGBE8 texel (4 B): m * 2^(e-136) is exactly the f32 radiant produced, so the
        // f64 value equals the reference's `color.r as f64` (verified per texel at upload).
        const uint32_t t = sc.hdri_rgbe[k];
        const uint32_t e = t >> 24;
        const double sc2 = e ? ldexp(1.0, (int)e - 136) : 0.0;
        return mk((double)(t & 0xffu) * sc2, (double)((t >> 8) & 0xffu) * sc2, (double)((t >> 16) & 0xffu) * sc2);
    }
    const float* px = sc.hdri + k * 3;
    return mk((double)px[0], (double)px[1], (double)px[2]);
}

__device__ __forceinline__ d3 checker(const DMaterial& m, d3 p) {  // texture.rs:58-70
    int32_t xi = sat_i32(floor(m.param * p.x));
    int32_t yi = sat_i32(floor(m.param * p.y));
    int32_t zi = sat_i32(floor(m.param * p.z));
    int32_t s = (int32_t)((uint32_t)xi + (uint32_t)yi + (uint32_t)zi);
    return (s % 2 == 0) ? ld3(m.a) : ld3(m.b);
}

// One shading lane: a miss (Camera::sample_background, camera.rs:201,228-233) or a hit
// (the HitRecord, then Material::emitted / scatter, material.rs).  cont = 1: the path
// continues from p along dir with attenuation col; cont = 0: it ends with radiance col
// (sky or emitted colour; 0 for an absorbed ray).
struct ShadeOut {
    d3 col, dir;
    uint32_t cont;
};

// Written as stages every shading lane passes through together, whatever its case, so
// a wave holding several cases pays once for the work they share instead of once per
// divergent branch: one unit() for the first normalisation (the rotated sky direction,
// the Lambertian ONB's w, the metal reflection, the dielectric's unit direction), one
// sqrt and division for the second (the ONB's v axis, random_unit_vector, and the
// dielectric's sin θ), one sqrt for the third (the cosine direction's unit, refract's
// parallel part), and one RNG draw for the Lambertian's r1 and the dielectric's Schlick
// draw.  Every lane evaluates exactly the reference's expressions on the same operands
// in the same order; only which lanes issue an instruction together changes.
// A hit lane's ray.o becomes the hit point p (the next ray's origin) as soon as p is
// known: nothing after the HitRecord reads the old origin, and p need not stay live.
template <bool PLAIN, bool SPH, bool GEN>
__device__ __forceinline__ ShadeOut shade(const DevScene& sc, Ray& ray, double t, uint32_t hit_ref,
                                          uint32_t hit_inst, uint64_t& rng, unsigned long long* cnt,
                                          uint32_t hit_outer = GS_REF_NONE) {
    const double PI = 3.14159265358979323846;
    ShadeOut o;
    o.cont = 0;
    o.col = mk(0.0, 0.0, 0.0);
    o.dir = mk(0.0, 0.0, 0.0);
    const bool miss = hit_ref == GS_REF_NONE;
    HitRec h;
    h.p = h.n = mk(0.0, 0.0, 0.0);
    h.u = h.v = 0.0;
    h.front = false;
    uint32_t kind = 0;  // 0: a miss
    const DMaterial* m = sc.mats;
    if (!miss) {
        atomicAdd(&cnt[C_HITS], 1ull);
        h = PLAIN ? reconstruct_sphere<false>(sc, ray, t, hit_ref)
            : SPH ? reconstruct_sphere<true>(sc, ray, t, hit_ref) : reconstruct<GEN>(sc, ray, t, hit_ref, hit_inst, hit_outer);
        m = &sc.mats[h.mat];
        kind = m->kind;
        ray.o = h.p;
    }
    const bool lamb = kind >= DM_LAMB_SOLID && kind <= DM_LAMB_TEX;  // material.rs:45-68
    const bool metal = kind == DM_METAL;                              // :87-102
    const bool diel = kind == DM_DIELECTRIC;                          // :123-148
    const bool iso = !PLAIN && (kind == DM_ISO_SOLID || kind == DM_ISO_TEX);  // :185-196
    const bool sky = miss && sc.bg.kind != GS_BG_SOLID;

    // albedo / emitted colour (texture.rs:27-95): one texture_value call site for every kind
    if (!PLAIN && (kind == DM_LAMB_TEX || kind == DM_LIGHT_TEX || kind == DM_ISO_TEX)) {
        o.col = texture_value(sc, m->texture, h.u, h.v, h.p, cnt);
    } else if (kind == DM_LAMB_CHECKER) {
        o.col = checker(*m, h.p);
    } else if (kind == DM_DIELECTRIC) {
        o.col = mk(1.0, 1.0, 1.0);
    } else if (!miss) {
        o.col = ld3(m->a);
    } else if (!sky) {
        o.col = ld3(sc.bg.color);
    }

    // stage 1: the first normalisation
    d3 v1 = mk(1.0, 0.0, 0.0);
    if (sky) {
        const double* R = sc.bg.rot;
        const d3 dir = ray.d;
        v1 = mk(dir.x * R[0] + dir.y * R[1] + dir.z * R[2], dir.x * R[3] + dir.y * R[4] + dir.z * R[5],
                dir.x * R[6] + dir.y * R[7] + dir.z * R[8]);
    } else if (lamb) {
        v1 = h.n;  // OrthonormalBasis::new (ONB.rs:10-23): w = unit(n)
    } else if (metal) {
        v1 = reflect(ray.d, h.n);
    } else if (diel) {
        v1 = ray.d;
    }
    const d3 u1 = unit(v1);

    // stage 2: the sky texel; the second vector to normalise (or sin θ's argument)
    d3 v2 = mk(1.0, 0.0, 0.0);
    double q2 = 1.0, ri = 0.0, cos_theta = 0.0;
    if (sky) {
        o.col = hdri_texel(sc, u1, cnt);
    } else if (lamb) {
        const d3 a = fabs(u1.x) > 0.9 ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
        v2 = cross(u1, a);
        q2 = len2(v2);
    } else if (metal || iso) {  // random_unit_vector (util.rs:18-29)
#pragma unroll 1
        for (;;) {
            double x = wy_f64(rng) * 2.0 + -1.0;
            double y = wy_f64(rng) * 2.0 + -1.0;
            double z = wy_f64(rng) * 2.0 + -1.0;
            v2 = mk(x, y, z);
            q2 = len2(v2);
            if (q2 < 1.0) break;
        }
    } else if (diel) {
        ri = h.front ? 1.0 / m->param : m->param;
        cos_theta = fmin(dot(neg(u1), h.n), 1.0);
        q2 = 1.0 - cos_theta * cos_theta;
    }
    const double r2v = sqrt(q2);  // |v2|, or the dielectric's sin θ
    d3 u2 = v2;
    if (lamb || metal || iso) u2 = divs(v2, r2v);

    // stage 3: the scattered direction
    double rd = 0.0;  // the first draw: the Lambertian's r1, the dielectric's Schlick draw
    if (lamb || diel) rd = wy_f64(rng);
    d3 w3 = mk(0.0, 0.0, 0.0), n3 = h.n;
    double q3 = 1.0;
    bool third = false;  // the lane finishes with the stage-3 sqrt
    if (lamb) {
        // random_cosine_direction (util.rs:48-60), r2^(1/4) quirk kept; ONB transform
        const d3 vv = u2;
        const d3 uu = cross(u1, vv);
        double r1 = rd;
        double r2 = wy_f64(rng);
        double phi = 2.0 * PI * r1;
        double r2s = sqrt(r2);
        double sp, cp;
        sincos(phi, &sp, &cp);
        double q = sqrt(r2s);
        d3 cd = mk(cp * q, sp * q, sqrt(1.0 - r2));
        w3 = add(add(muls(uu, cd.x), muls(vv, cd.y)), muls(u1, cd.z));
        q3 = len2(w3);
        third = true;
        o.cont = 1;
    } else if (metal) {
        const d3 reflected = add(u1, muls(u2, m->param));
        if (dot(reflected, h.n) > 0.0) {
            o.dir = reflected;
            o.cont = 1;
        } else {
            o.col = mk(0.0, 0.0, 0.0);  // absorbed
        }
    } else if (iso) {
        o.dir = u2;
        o.cont = 1;
    } else if (diel) {
        const d3 ud = u1;
        double sin_theta = r2v;
        bool cannot_refract = ri * sin_theta > 1.0;
        double r0 = (1.0 - ri) / (1.0 + ri);
        r0 = r0 * r0;
        double x = 1.0 - cos_theta;
        double x2 = x * x;
        double x4 = x2 * x2;
        double refl = r0 + (1.0 - r0) * (x * x4);  // powi(x, 5) as LLVM expands it
        bool fresnel = refl > rd;
        if (cannot_refract || fresnel) {
            o.dir = reflect(ud, h.n);
        } else {  // refract (vec3.rs:57-62)
            double ct = fmin(dot(h.n, neg(ud)), 1.0);
            w3 = muls(add(ud, muls(h.n, ct)), ri);
            q3 = fabs(1.0 - len2(w3));
            third = true;
        }
        o.cont = 1;
    }
    if (third) {
        const double r3 = sqrt(q3);
        if (lamb) o.dir = divs(w3, r3);                    // unit(cosine direction)
        else o.dir = add(w3, muls(n3, -r3));               // r_out_perp + r_out_parallel
    }
    return o;
}

// ---- split shading (scenes with at most two of: sky, Lambertian, metal, dielectric,
// isotropic): one divergent branch per case, no select overhead.
// Camera::sample_background / HDRI::sample (camera.rs:228-233, 257-270).
__device__ GS_NOINLINE d3 background(const DevScene& sc, d3 dir, unsigned long long* cnt) {
    const gs_background& bg = sc.bg;
    if (bg.kind == GS_BG_SOLID) return ld3(bg.color);
    d3 rv = mk(dir.x * bg.rot[0] + dir.y * bg.rot[1] + dir.z * bg.rot[2],
               dir.x * bg.rot[3] + dir.y * bg.rot[4] + dir.z * bg.rot[5],
               dir.x * bg.rot[6] + dir.y * bg.rot[7] + dir.z * bg.rot[8]);
    return hdri_texel(sc, unit(rv), cnt);
}

__device__ __forceinline__ d3 random_unit_vector(uint64_t& rng) {  // util.rs:18-29
    d3 v;
#pragma unroll 1
    for (;;) {
        double x = wy_f64(rng) * 2.0 + -1.0;
        double y = wy_f64(rng) * 2.0 + -1.0;
        double z = wy_f64(rng) * 2.0 + -1.0;
        v = mk(x, y, z);
        if (len2(v) < 1.0) break;
    }
    return unit(v);
}

// Material::emitted + Material::scatter (material.rs).  kind: 0 = path ends with
// `col` (emitted colour; 0 for an absorbed ray), 1 = continues along `dir` with
// attenuation `col`.
struct Scatter {
    d3 col, dir;
    uint64_t rng;
    uint32_t cont;
};

__device__ GS_NOINLINE Scatter scatter(const DevScene& sc, HitRec h, d3 in_dir, uint64_t rng,
                                        unsigned long long* cnt) {
    const DMaterial& m = sc.mats[h.mat];
    Scatter s;
    s.cont = 0;
    s.col = mk(0.0, 0.0, 0.0);
    s.dir = mk(0.0, 0.0, 0.0);
    const uint32_t kind = m.kind;
    if (kind <= DM_LAMB_TEX) {  // Lambertian :45-68
        s.col = kind == DM_LAMB_SOLID ? ld3(m.a)
              : kind == DM_LAMB_CHECKER ? checker(m, h.p)
                                        : texture_value(sc, m.texture, h.u, h.v, h.p, cnt);
        // OrthonormalBasis::new (ONB.rs:10-23)
        d3 w = unit(h.n);
        d3 a = fabs(w.x) > 0.9 ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
        d3 vv = unit(cross(w, a));
        d3 uu = cross(w, vv);
        // random_cosine_direction (util.rs:48-60), r2^(1/4) quirk kept
        const double PI = 3.14159265358979323846;
        double r1 = wy_f64(rng);
        double r2 = wy_f64(rng);
        double phi = 2.0 * PI * r1;
        double r2s = sqrt(r2);
        double sp, cp;
        sincos(phi, &sp, &cp);
        double q = sqrt(r2s);
        d3 cd = mk(cp * q, sp * q, sqrt(1.0 - r2));
        s.dir = unit(add(add(muls(uu, cd.x), muls(vv, cd.y)), muls(w, cd.z)));
        s.cont = 1;
    } else if (kind == DM_METAL) {  // :87-102
        d3 reflected = reflect(in_dir, h.n);
        reflected = add(unit(reflected), muls(random_unit_vector(rng), m.param));
        if (dot(reflected, h.n) > 0.0) {
            s.col = ld3(m.a);
            s.dir = reflected;
            s.cont = 1;
        }
    } else if (kind == DM_DIELECTRIC) {  // :123-148
        double ri = h.front ? 1.0 / m.param : m.param;
        d3 ud = unit(in_dir);
        double cos_theta = fmin(dot(neg(ud), h.n), 1.0);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        bool cannot_refract = ri * sin_theta > 1.0;
        double r0 = (1.0 - ri) / (1.0 + ri);
        r0 = r0 * r0;
        double x = 1.0 - cos_theta;
        double x2 = x * x;
        double x4 = x2 * x2;
        double refl = r0 + (1.0 - r0) * (x * x4);  // powi(x, 5) as LLVM expands it
        bool fresnel = refl > wy_f64(rng);
        s.dir = (cannot_refract || fresnel) ? reflect(ud, h.n) : refract(ud, h.n, ri);
        s.col = mk(1.0, 1.0, 1.0);
        s.cont = 1;
    } else if (kind == DM_ISO_SOLID || kind == DM_ISO_TEX) {  // Isotropic :185-196
        s.col = kind == DM_ISO_SOLID ? ld3(m.a) : texture_value(sc, m.texture, h.u, h.v, h.p, cnt);
        s.dir = random_unit_vector(rng);
        s.cont = 1;
    } else {  // DiffuseLight :165-169 (emits, never scatters)
        s.col = kind == DM_LIGHT_SOLID ? ld3(m.a) : texture_value(sc, m.texture, h.u, h.v, h.p, cnt);
    }
    s.rng = rng;
    return s;
}


// The placement pilot's count (GS_FEAT_VISITS): one atomic per distinct record among the
// wave's active lanes (every ray of a pilot tests the root and the records below it: one
// atomic per lane on those addresses serialised the pilot, 111 ms on MI355X C4).
// The lead lane is retired every round whatever the ballot returns, so the loop ends
// after at most 64 rounds even if the mask it starts from held a lane that is not active
// here (the round-3 stamps-build hang: DESIGN.md §7); a lane outside `same` but in `m`
// is then counted by nobody, which the pilot's tests would show as a miscount.
__device__ __forceinline__ void count_visit(uint32_t* counts, uint32_t idx) {
    uint64_t m = __builtin_amdgcn_ballot_w64(true);
#pragma unroll 1
    while (m != 0) {
        const uint32_t lead = (uint32_t)__builtin_ctzll(m);
        const uint32_t v = __builtin_amdgcn_readlane(idx, lead);
        const uint64_t same = __builtin_amdgcn_ballot_w64(idx == v);
        if ((threadIdx.x & 63u) == lead) atomicAdd(&counts[v], (uint32_t)__popcll(same));
        m &= ~(same | (1ull << lead));
    }
}

// Diagnostic build only (-DGS_STAMPS): per-wave shader-clock totals of the three loop
// phases, written to their own debug buffer (the d_item_visits pointer, reinterpreted
// as u64[3]) — never to an output.  The stamps' fences perturb scheduling, so only the
// shares are meaningful, not the absolute time.
#if defined(GS_STAMPS)
#define GS_STAMP(t) do { __builtin_amdgcn_sched_barrier(0); t = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
// Region timing inside divergent shading code: the first active lane adds the wave's
// elapsed clock to its wave's LDS slot (one count per wave, whatever the mask).
#define GS_REGION(k, t0) do { uint64_t t1_; GS_STAMP(t1_); \
    const uint64_t em_ = __builtin_amdgcn_read_exec(); \
    if (lane == (uint32_t)__builtin_ctzll(em_)) s_reg[(tid >> 6) * 16 + (k)] += t1_ - (t0); } while (0)
#else
#define GS_STAMP(t) do { } while (0)
#define GS_REGION(k, t0) do { } while (0)
#endif
// Diagnostic builds (-DGS_WATCHDOG=N; on in the stamps build): a wave whose traversal phase
// takes more than N passes, or whose loop more than 64 N iterations, prints every lane's
// state once (the first 4 such waves of the launch) and retires its lanes, so a loop that
// does not end names itself instead of running into the caller's time limit.
#if defined(GS_STAMPS) && !defined(GS_WATCHDOG)
#define GS_WATCHDOG (1 << 20)
#endif
#ifdef GS_WATCHDOG
__device__ unsigned int g_wd_trips;
#endif


// Per-lane pixel state lives in LDS ([field][lane], conflict-free), touched once per
// path; the mirror of the tree's top records follows it.
enum { L_CSR = 0, L_CSG, L_CSB, L_LSUM, L_LSQ, L_SCOUNT, L_ND };
enum { L_ITEM = 0, L_PIX, L_BLEFT, L_SAMPLE, L_DEPTH, L_HINST, L_NI };  // (sample, depth, hit
// instance: per-path state touched once per bounce, kept out of the traversal loop's VGPRs)

// Lane state plus the block's 64-bit counters (C_N of them, 128 B).  There is no static
// LDS: the dynamic LDS then starts at address 0, so a node's LDS address is its byte
// offset itself (node links are pre-shifted, below).
#ifdef GS_STAMPS
#define GS_STAMP_LDS ((GS_BLOCK / 64) * 16 * 8)
#else
#define GS_STAMP_LDS 0
#endif
// Fixed-spp (chunked) launches never reach the stop test, so their lanes keep only the
// three colour sums: the 24 KiB of Σlum / Σlum² / sample-count slots go to the mirror.
enum { L_ND_CHUNKED = L_LSUM };
// Media / nested-BVH kernels keep the path throughput (Tr, Tg, Tb: read and written only
// by the shade pass) in three more f64 lane fields (before those), out of the registers their
// leaf tests need (round 3: with them in VGPRs these instantiations spilled 52-76 B/lane).
// (not the placement pilot's counting kernel: it launches with the scene's own lane layout)
__host__ __device__ constexpr bool t_in_lds(int feat) {
    return (feat & (GS_FEAT_MEDIA | GS_FEAT_NESTED)) != 0 && (feat & GS_FEAT_VISITS) == 0;
}
// ... and, in kernels that walk BVHs under instances, the lane's save slots (the top-level
// ray, the return link and -- the general kernel -- a hit's outer chain, while the lane walks
// such a tree) in 7 or 8 more f64 fields at the end when the block's LDS has room for them
// beside the whole mirror (KArgs::nest_lds): written at each tree entry, read at its THR_RET.
// Else in global memory (KParams::nest_save, slot-major; also the pilot's counting kernel).
// Off by default: the one scene it helps by traffic (final_scene: 9x fewer fabric writes) lost
// 5% to the mirror records the slots displace, and the run-time choice between the two homes
// cost final_scene 2% more in the kernel that has both (profiles/r06/ab_nest_save_lds.txt).
#ifndef GS_NEST_SAVE_LDS
#define GS_NEST_SAVE_LDS 0
#endif
__host__ __device__ constexpr uint32_t nest_save_lds(int feat) {
    return (GS_NEST_SAVE_LDS && (feat & GS_FEAT_NESTED) != 0 && (feat & GS_FEAT_VISITS) == 0)
               ? ((feat & GS_FEAT_GENERAL) ? 8u : 7u)
               : 0u;
}
__host__ __device__ constexpr uint32_t lane_nd(bool chunked, int feat) {
    return (chunked ? (uint32_t)L_ND_CHUNKED : (uint32_t)L_ND) + (t_in_lds(feat) ? 3u : 0u);
}
// ... and the hit primitive's ref (written by leaf tests, read by the shade pass) in one
// more u32 field, L_HREF.
enum { L_HREF = L_NI };
// ... and, in kernels that walk BVHs under instances (GS_FEAT_NESTED), the instance chain
// whose tree the lane walks (GS_REF_NONE at the top level) in one more, L_NINST (not the
// placement pilot's: it launches with the scene's own lane layout and keeps it in a register).
__host__ __device__ constexpr bool ninst_in_lds(int feat) {
    return (feat & GS_FEAT_NESTED) != 0 && (feat & GS_FEAT_VISITS) == 0;
}
__host__ __device__ constexpr uint32_t lane_ninst(int feat) { return (uint32_t)L_NI + (t_in_lds(feat) ? 1u : 0u); }
__host__ __device__ constexpr uint32_t lane_ni(int feat) { return lane_ninst(feat) + (ninst_in_lds(feat) ? 1u : 0u); }
__host__ __device__ constexpr size_t lane_lds_bytes(bool chunked, int feat, uint32_t nsave = 0) {
    return (size_t)GS_BLOCK * ((lane_nd(chunked, feat) + nsave) * 8 + lane_ni(feat) * 4) + 128 + GS_STAMP_LDS;
}

template <int FEAT>
#ifdef GS_NUM_VGPR
__attribute__((amdgpu_num_vgpr(GS_NUM_VGPR)))
#endif
__global__ __launch_bounds__(GS_BLOCK, GS_MIN_WAVES) void gs_render_kernel(KArgs A) {
    extern __shared__ __align__(16) uint8_t smem[];
    // An empty batch round (adaptive settings: no active pixel left in this segment) has no
    // item to hand out: return before the mirror copy.
    if ((!(FEAT & GS_FEAT_FIXED) || (FEAT & GS_FEAT_RSPLIT)) && A.P->rounds && A.P->n_items == 0) return;

    // The records a ray most likely tests (placed first by the host) are mirrored in LDS;
    // a lane whose node / leaf index is below lds_nodes / lds_leaves reads it from there
    // (ds_read), the rest from global memory.  The node mirror starts the dynamic LDS, so
    // a node's LDS address is cur << 5 plus a constant the ds_read offset absorbs.
    uint8_t* s_nodes = smem;
    uint8_t* s_leaves = s_nodes + (size_t)A.lds_nodes * sizeof(TNode);
    uint8_t* s_quads = s_leaves + (size_t)A.lds_leaves * sizeof(TLeaf);
    {
        const uint4* src = reinterpret_cast<const uint4*>(A.tnodes);
        uint4* dst = reinterpret_cast<uint4*>(s_nodes);
        for (uint32_t k = threadIdx.x; k < A.lds_nodes * 2u; k += GS_BLOCK) dst[k] = src[k];
        src = reinterpret_cast<const uint4*>(A.tleaves);
        dst = reinterpret_cast<uint4*>(s_leaves);
        for (uint32_t k = threadIdx.x; k < A.lds_leaves * 3u; k += GS_BLOCK) dst[k] = src[k];
        src = reinterpret_cast<const uint4*>(A.tquads);
        dst = reinterpret_cast<uint4*>(s_quads);
        for (uint32_t k = threadIdx.x; k < A.lds_quads * 8u; k += GS_BLOCK) dst[k] = src[k];
        src = reinterpret_cast<const uint4*>(A.cubes);
        dst = reinterpret_cast<uint4*>(s_quads + (size_t)A.lds_quads * sizeof(TQuad));
        for (uint32_t k = threadIdx.x; k < A.lds_cubes * (GS_CUBE_DOUBLES / 2); k += GS_BLOCK) dst[k] = src[k];
    }
    uint8_t* s_cubes = s_quads + (size_t)A.lds_quads * sizeof(TQuad);
    const QuadSrc qs{s_quads, A.tquads, A.lds_quads, s_cubes, A.lds_cubes};
    // Per-lane pixel / path state after the mirror: [L_ND][GS_BLOCK] f64, [L_NI][GS_BLOCK] u32.
    double* s_d = (double*)(s_cubes + (size_t)A.lds_cubes * (GS_CUBE_DOUBLES * 8));
    uint32_t* s_i = (uint32_t*)(s_d + A.lane_nd * GS_BLOCK);
    unsigned long long* s_cnt = (unsigned long long*)(s_i + lane_ni(FEAT) * GS_BLOCK);
#ifdef GS_STAMPS
    unsigned long long* s_reg = s_cnt + 16;  // [(GS_BLOCK / 64) * 16]: shade regions 0-4, leaf kinds 8-15
    if (threadIdx.x < (GS_BLOCK / 64) * 16) s_reg[threadIdx.x] = 0;
#endif
    if (threadIdx.x < GS_CNT_SLOTS) s_cnt[threadIdx.x] = 0;
    __syncthreads();

    const KParams* __restrict__ P = A.P;
    const DevScene& sc = P->sc;
    const gs_camera& cam = P->cam;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t tid = threadIdx.x;
    const uint64_t flushers = __builtin_amdgcn_ballot_w64(tid < GS_CNT_SLOTS);  // the counters' flushing lanes
    const double tmin = 0.001;
    constexpr int kUnroll = unroll_steps(FEAT);  // node steps of an unrolled node pass
    // Every top-level leaf a stationary sphere: no instance is ever hit, so the hit's
    // instance (lane state L_HINST) stays GS_REF_NONE from the kernel's start.
    constexpr bool kSphLeaf = (FEAT & GS_FEAT_SPHLEAF) != 0;
    // A fixed-spp chunked launch (the host's choice, kernel_for): P->chunk != 0, no rounds, no
    // per-sample colours, max_depth > 0 -- a camera ray is always due when advance() runs.
    constexpr bool kFixed = (FEAT & GS_FEAT_FIXED) != 0;
    // ... or a batch round's split items in that form (GS_FEAT_RSPLIT: per-sample colours)
    constexpr bool kRsplit = kFixed && (FEAT & GS_FEAT_RSPLIT) != 0;
    constexpr bool kGeneral = (FEAT & GS_FEAT_GENERAL) != 0;
    // (t_in_lds kernels: the throughput's three fields first, at fixed offsets)
#define LD(k) s_d[((k) + (t_in_lds(FEAT) ? 3 : 0)) * GS_BLOCK + tid]
#define LI(k) s_i[(k) * GS_BLOCK + tid]
    if constexpr (kSphLeaf) LI(L_HINST) = GS_REF_NONE;
    // GS_FEAT_NESTED: the instance chain whose BVH the lane walks (GS_REF_NONE: the top level)
    constexpr bool kNested = (FEAT & GS_FEAT_NESTED) != 0;
    uint32_t ninst_ = GS_REF_NONE;
#define LNINST (*(ninst_in_lds(FEAT) ? &s_i[lane_ninst(FEAT) * GS_BLOCK + tid] : &ninst_))
    if constexpr (kNested) LNINST = GS_REF_NONE;
    // the lane's nested-walk save slot k: the last f64 lane fields (nest_save_lds), else the
    // slot-major global array (slot k of every lane of the grid contiguous)
    double* const s_save = s_d + (size_t)(A.lane_nd - A.nest_lds) * GS_BLOCK + tid;
    const size_t g_lanes = (size_t)gridDim.x * GS_BLOCK;
#define NSAVE(k)                                                                                   \
    (*(nest_save_lds(FEAT) && A.nest_lds ? &s_save[(size_t)(k) * GS_BLOCK]                         \
                                         : &P->nest_save[(size_t)(k) * g_lanes + (size_t)blockIdx.x * GS_BLOCK + tid]))

    uint32_t st = S_NEED;
    bool qdone = false;
    uint32_t res_base = 0, res_cnt = 0;  // the wave's reserve of claimed items (wave-uniform)
    // path state (registers)
    uint64_t rng = 0;
    // path throughput: registers, or the last three f64 lane fields (t_in_lds)
    constexpr bool kTLds = t_in_lds(FEAT);
    double Tr_ = 1, Tg_ = 1, Tb_ = 1;
#define GS_TP(reg, k) (*(kTLds ? &s_d[(k) * GS_BLOCK + tid] : &(reg)))
#define Tr GS_TP(Tr_, 0)
#define Tg GS_TP(Tg_, 1)
#define Tb GS_TP(Tb_, 2)
    Ray ray;
    ray.o = mk(0, 0, 0);
    ray.d = mk(0, 0, 0);
    ray.time = 0;
    RayCert rc{};  // the ray in the certified f32 slab test's terms (geometry.hpp)
    // traversal state
    uint32_t cur = THR_END, hit_ref_ = GS_REF_NONE;
    // the hit primitive's ref: a register, or the lane's L_HREF field (t_in_lds kernels)
    uint32_t& hit_ref = kTLds ? s_i[L_HREF * GS_BLOCK + tid] : hit_ref_;
    double closest = 0.0;
    float closest32 = 0.0f;  // f32(closest)
    const float tmin32 = 0.001f;  // f32(tmin)
    bool fast = false;  // a cert ray: nodes take box_cert (geometry.hpp)
    // The lane has a new ray in `ray` whose traversal state begin_ray has not set up yet:
    // camera rays (advance) and scattered rays (shade) meet in one begin_ray per phase, so
    // a wave pays for it once, not once per branch.
    bool fresh = false;
    // hot counters kept in registers, flushed per pixel
    uint32_t c_nodes = 0, c_sph = 0;  // (per lane: one VALU add beat a 64-bit SALU wave count)

    auto begin_ray = [&]() {
        // AABB::hit's `1.0 / ray.direction[axis]` (AABB.rs:64), hoisted per ray for the certified
        // f32 test's constants (rcp_cert: within 2^-52 of it; the f64 test takes inv_of's exact one)
        const d3 inv = inv_cert(ray.d);
        fast = A.cert_boxes && cert_ray_ok(ray.o, inv);
        rc = make_cert(ray.o, inv);
        cur = A.root;  // the root record's link (THR_*)
        closest = 1.7976931348623157e308;  // f64::MAX (camera.rs:177)
        closest32 = __builtin_inff();
        hit_ref = GS_REF_NONE;
        if constexpr (!kSphLeaf) LI(L_HINST) = GS_REF_NONE;  // (sphere-only trees: never set)
        atomicAdd(&s_cnt[C_RAYS], 1ull);
    };

    // camera.rs:142-146 for one finished sample of colour L
    auto add_sample = [&](double Lr, double Lg, double Lb) {
        if (kRsplit || (!kFixed && P->per_sample)) {  // batch rounds: the sample's colour, summed in order by the combine
            double* o = P->partial + (size_t)LI(L_ITEM) * 3;
            st_partial(o, Lr, Lg, Lb);
            LI(L_ITEM) += GS_ROUND_PIXEL_MAJOR ? 1u : P->seg_n;
        } else {
            LD(L_CSR) += Lr;
            LD(L_CSG) += Lg;
            LD(L_CSB) += Lb;
        }
        if (!kFixed && !P->chunk) {  // a chunk never reaches the stop test: Σlum, Σlum² unused
            double lum = 0.299 * Lr + 0.587 * Lg + 0.144 * Lb;
            LD(L_LSUM) += lum;
            LD(L_LSQ) += lum * lum;
        }
        LI(L_SAMPLE) += 1u;
        LI(L_BLEFT) -= 1u;
    };

    // Start samples until one needs tracing or the pixel is finished:
    // leaves st = S_TRACE (ray ready) or S_NEED (pixel written).
    // End of a chunk: its Σrgb, summed per pixel by gs_combine_kernel.
    // The lane's node-visit and sphere-test counts go to the block's counters at the end of
    // the kernel -- or at an item's end when the launch records per-item visits (the tile
    // plan's pilot), or before a count could overflow.  (Flushing at every item's end ran
    // the compiler's lane-serial reduction loop of two 64-bit atomics per chunk.)
    auto flush_counts = [&]() {
        atomicAdd(&s_cnt[C_NODES], (unsigned long long)c_nodes);
        atomicAdd(&s_cnt[C_SPH], (unsigned long long)c_sph);
        c_nodes = 0;
        c_sph = 0;
    };
    // a stationary-sphere test: a lane count (flushed with c_nodes), or in t_in_lds kernels
    // a wave-aggregated LDS atomic, as prim_test counts the other kinds (no register kept)
    auto count_sph = [&]() __attribute__((always_inline)) {
        if constexpr (kTLds) atomicAdd(&s_cnt[C_SPH], 1ull);
        else c_sph++;
    };
    auto end_chunk = [&]() {
        const uint32_t item = LI(L_ITEM);
        if (!kRsplit && (kFixed || !P->per_sample)) {
            double* o = P->partial + (size_t)item * 3;
            st_partial(o, LD(L_CSR), LD(L_CSG), LD(L_CSB));
        }
#if !defined(GS_STAMPS) && !defined(GS_CERT_CHECK)  // (those builds use item_visits as their record buffer)
        if (P->item_visits) {  // (the item's packed pixel, from its chunk-major sum slot)
            const uint32_t k = item < P->fine_base ? item % P->fine_px
                                                   : P->fine_px + (item - P->fine_base) % (P->capacity - P->fine_px);
            atomicAdd(&P->item_visits[k], c_nodes);
            flush_counts();
        }
#endif
        if ((c_nodes | c_sph) >= (1u << 30)) flush_counts();
        st = S_NEED;
    };

    auto advance = [&]() {
#pragma unroll 1
        for (;;) {
            // (fixed-spp launches: the shade pass ends a chunk at its last sample, so a lane
            // here always has a sample left and max_depth > 0 -- straight to get_ray)
            if (!kFixed && LI(L_BLEFT) == 0) {
                if (P->chunk) {
                    end_chunk();
                    return;
                }
                // end of a batch (camera.rs:149-164)
                const double scount = LD(L_SCOUNT), lsum = LD(L_LSUM), lsq = LD(L_LSQ);
                const double confidence_sq = P->ss.confidence * P->ss.confidence;
                const double tolerance_sq = P->ss.tolerance * P->ss.tolerance;
                double mean = lsum / scount;
                double variance_sq = 1.0 / (scount - 1.0) * (lsq - lsum * lsum / scount);
                double convergence_sq = confidence_sq * variance_sq / scount;
                bool stop = convergence_sq < (mean * mean * tolerance_sq);
                if (!stop) stop = (uint32_t)sat_u64(scount, 4294967295.0, 4294967295ull) > P->ss.max_samples;
                if (stop) {
                    const uint32_t item = LI(L_ITEM);
                    const size_t oi = P->direct ? (size_t)LI(L_PIX) : (size_t)item;
                    const double cr = LD(L_CSR) / scount, cg = LD(L_CSG) / scount, cb = LD(L_CSB) / scount;
                    if (P->out) {
                        float* o = P->out + oi * 3;
                        o[0] = (float)cr;
                        o[1] = (float)cg;
                        o[2] = (float)cb;
                    }
                    if (P->out8) {
                        uint8_t* o8 = P->out8 + oi * 3;
                        o8[0] = color_byte(cr);
                        o8[1] = color_byte(cg);
                        o8[2] = color_byte(cb);
                    }
                    atomicAdd(&s_cnt[C_PIX], 1ull);
#if !defined(GS_STAMPS) && !defined(GS_CERT_CHECK)
                    if (P->item_visits) {
                        P->item_visits[item] = c_nodes;
                        flush_counts();
                    }
#endif
                    if ((c_nodes | c_sph) >= (1u << 30)) flush_counts();
                    st = S_NEED;
                    return;
                }
                if (P->rounds) {  // batch rounds: the sums wait for the next round, maybe in another lane
                    const uint32_t item = LI(L_ITEM);
                    double* ps = P->pstate + (size_t)item * 5;
                    ps[0] = LD(L_CSR);
                    ps[1] = LD(L_CSG);
                    ps[2] = LD(L_CSB);
                    ps[3] = lsum;
                    ps[4] = lsq;
                    P->next_active[atomicAdd(&P->round_counts[P->round + 1u], 1u)] = item;
                    if ((c_nodes | c_sph) >= (1u << 30)) flush_counts();
                    st = S_NEED;
                    return;
                }
                LD(L_SCOUNT) = scount + (double)P->ss.batch_size;
                LI(L_BLEFT) = P->ss.batch_size;
            }
            // Camera::get_ray (camera.rs:204-221) on the seeded stream of this sample
            const uint32_t pix = LI(L_PIX);
            const uint32_t pj = udiv(pix, P->u_w), pi = pix - pj * (uint32_t)cam.image_width;
            rng = stream_seed(P->seed, pix, LI(L_SAMPLE));
            atomicAdd(&s_cnt[C_PATHS], 1ull);
            double offx = wy_f64(rng) - 0.5;
            double offy = wy_f64(rng) - 0.5;
            double si = (double)pi + offx, sj = (double)pj + offy;
            d3 ps = add(add(ld3(cam.starting_pixel_pos), muls(ld3(cam.pixel_delta_u), si)),
                        muls(ld3(cam.pixel_delta_v), sj));
            d3 org;
            if (cam.defocus_angle <= 0.0) {
                org = ld3(cam.center);
            } else {  // defocus_disk_sample (camera.rs:223-226, util.rs:36-46)
                double dx, dy;
#pragma unroll 1
                for (;;) {
                    dx = wy_f64(rng) * 2.0 + -1.0;
                    dy = wy_f64(rng) * 2.0 + -1.0;
                    if (dx * dx + dy * dy + 0.0 * 0.0 < 1.0) break;
                }
                org = add(add(ld3(cam.center), muls(ld3(cam.defocus_disk_u), dx)), muls(ld3(cam.defocus_disk_v), dy));
            }
            ray.o = org;
            ray.d = sub(ps, org);
            ray.time = wy_f64(rng);
#if defined(GS_DIAG_DUP) && (GS_DIAG_DUP & 4)
            {  // cost probe: get_ray's draws and arithmetic twice, plus begin_ray's reciprocals
                uint64_t g2 = stream_seed(P->seed, pix, LI(L_SAMPLE));
                asm volatile("" : "+v"(g2));
                double ox2 = wy_f64(g2) - 0.5, oy2 = wy_f64(g2) - 0.5;
                d3 ps2 = add(add(ld3(cam.starting_pixel_pos), muls(ld3(cam.pixel_delta_u), (double)pi + ox2)),
                             muls(ld3(cam.pixel_delta_v), (double)pj + oy2));
                d3 org2 = ld3(cam.center);
                if (cam.defocus_angle > 0.0) {
                    double dx, dy;
#pragma unroll 1
                    for (;;) {
                        dx = wy_f64(g2) * 2.0 + -1.0;
                        dy = wy_f64(g2) * 2.0 + -1.0;
                        if (dx * dx + dy * dy + 0.0 * 0.0 < 1.0) break;
                    }
                    org2 = add(add(ld3(cam.center), muls(ld3(cam.defocus_disk_u), dx)), muls(ld3(cam.defocus_disk_v), dy));
                }
                const d3 d2 = sub(ps2, org2);
                const double tm2 = wy_f64(g2);
                const d3 inv2 = mk(1.0 / d2.x, 1.0 / d2.y, 1.0 / d2.z);
                asm volatile("" ::"v"(inv2.x), "v"(inv2.y), "v"(inv2.z), "v"(tm2), "v"(org2.x), "v"(org2.y), "v"(org2.z));
            }
#endif
            Tr = Tg = Tb = 1.0;
            LI(L_DEPTH) = cam.max_depth;
            if (kFixed || cam.max_depth > 0) {
                fresh = true;  // begin_ray by the caller
                st = S_TRACE;
                return;
            }
            add_sample(0.0, 0.0, 0.0);  // ray_color(ray, 0) = 0 (camera.rs:175)
        }
    };

    uint64_t ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, acc_refill = 0, acc_trav = 0, acc_shade = 0;
    uint64_t acc_node = 0, acc_leaf = 0;  // stamps build: wave clock in node / leaf passes
    uint64_t dist_ref = 0, dist_kind = 0;  // stamps build: distinct leaf refs / ref kinds per leaf pass
    uint64_t dist_bad = 0;                 // stamps build: those counts' loops that did not converge
    uint64_t it_all = 0, it_node = 0, it_leaf = 0, ln_node = 0, ln_leaf = 0, it_shade = 0, ln_shade = 0;
    uint64_t it_adv = 0, ln_adv = 0;  // stamps build: camera-ray (advance) executions and their lanes
    // stamps build: node steps (lanes) from global memory; wave node steps with any active lane,
    // with any lane reading its record from global memory; active lanes over those steps
    uint64_t d_gvis = 0, d_wsteps = 0, d_wsteps_g = 0, d_wlanes = 0;
#ifdef GS_WATCHDOG
    uint32_t wd_loop = 0;
    // prints the lane's state (once per tripped wave, the launch's first 4) and retires the lane
    auto wd_trip = [&](const char* where, uint32_t count) {
        uint32_t k = 0;
        if (lane == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) k = atomicAdd(&g_wd_trips, 1u);
        k = __builtin_amdgcn_readfirstlane(k);
        if (k < 4)
            printf("GS_WATCHDOG %s n=%u block=%u wave=%u lane=%u st=%u cur=%08x fast=%d closest=%g hit_ref=%08x "
                   "depth=%u bleft=%u item=%u sample=%u res_cnt=%u qdone=%d o=(%g %g %g) d=(%g %g %g)\n",
                   where, count, (unsigned)blockIdx.x, (unsigned)(tid >> 6), lane, st, cur, (int)fast, closest,
                   (uint32_t)hit_ref, LI(L_DEPTH), LI(L_BLEFT), LI(L_ITEM), LI(L_SAMPLE), res_cnt, (int)qdone, ray.o.x,
                   ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z);
        st = S_DONE;
        cur = THR_END;
        fresh = false;
        qdone = true;
    };
#endif
#pragma unroll 1
    for (;;) {
        // ---------------------------------------------------------- refill
        GS_STAMP(ts0);
#ifdef GS_WATCHDOG
        if (++wd_loop > 64u * (uint32_t)GS_WATCHDOG) {
            wd_trip("loop", wd_loop);
            break;
        }
#endif
        // Refill and camera rays: lanes without an item take one (S_NEED -> S_CAM), then every
        // lane whose next sample needs a camera ray -- a new item's first, or the next sample
        // after the shade pass finished one -- runs advance() together, once per loop
        // iteration (the wave pays for get_ray once, not once per refill and once per shade).
        // advance() hands back S_TRACE, or S_NEED when an item ends there (adaptive settings,
        // max_depth 0), which sends the lane round once more.
#pragma unroll 1
        for (;;) {
        uint64_t need = __builtin_amdgcn_ballot_w64(st == S_NEED);
#pragma unroll 1
        while (need != 0 && !qdone) {
            // Lanes take items from the wave's reserve; an empty reserve is refilled with
            // `claim` items by one atomic (a contended device-scope atomic per refill round
            // cost ~5% of wave time with 8-sample items).  Items are independent, so who
            // runs which one changes nothing in the result.
            if (res_cnt == 0) {
                const uint32_t leader = (uint32_t)__ffsll((long long)need) - 1;
                uint32_t base = 0;
                const uint32_t cl = res_base >= P->fine_base ? P->claim_fine : P->claim;
                if (lane == leader) base = atomicAdd(P->queue, cl);
                base = __builtin_amdgcn_readfirstlane(__shfl(base, leader));
                if (base >= P->n_items) {
                    qdone = true;
                    break;
                }
                res_base = base;
                res_cnt = min(cl, P->n_items - base);
            }
            const uint32_t n = (uint32_t)__popcll(need);
            const uint32_t take = min(n, res_cnt);
            const uint32_t base = res_base;
            res_base += take;
            res_cnt -= take;
            const uint32_t tile_px = (uint32_t)(P->tile_w * P->tile_h);
            const bool blocked8 = (P->tile_w % 8 == 0) && (P->tile_h % 8 == 0);
            // set bits of `need` below this lane (v_mbcnt: no 64-bit lane mask kept live)
            // (media / nested / sphere-only kernels; the others keep the popcount of the
            // masked ballot: C3 +0.6%, C5 +1.2%, C4 -0.3% the other way round)
#ifndef GS_RANK_MBCNT
#define GS_RANK_MBCNT ((FEAT & (GS_FEAT_MEDIA | GS_FEAT_NESTED | GS_FEAT_SPHLEAF)) != 0)
#endif
            const uint32_t rank =
                GS_RANK_MBCNT ? __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u))
                              : (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
            if (st == S_NEED && rank < take) {
                const uint64_t q = (uint64_t)base + (uint64_t)rank;
                if (q >= P->n_items) {
                    st = S_DONE;
                } else {
                    // work order: 8x8 blocks inside each tile (coherent primary rays), a
                    // pixel's chunks adjacent
                    const uint32_t q32 = (uint32_t)q;  // q < n_items < 2^32
                    const bool fine = q32 >= P->fine_base;
                    const uint32_t cpp = fine ? P->fine_cpp : P->cpp, csz = fine ? P->fine_chunk : P->chunk;
                    const uint32_t qr = fine ? q32 - P->fine_base : q32;
                    const uint32_t pr = udiv(qr, fine ? P->u_fcpp : P->u_cpp), ck = qr - pr * cpp;
                    uint32_t slot, x, y;
                    if (kRsplit || (!kFixed && P->rounds)) {  // batch rounds: the packed pixel of active entry pr
                        const uint32_t it = P->active[P->seg_base + pr];
                        slot = udiv(it, P->u_tpx);
                        const uint32_t w = it - slot * tile_px;
                        y = udiv(w, P->u_tw);
                        x = w - y * (uint32_t)P->tile_w;
                    } else {
                        const uint32_t pq = fine ? P->fine_px + pr : pr;
                        slot = udiv(pq, P->u_tpx);
                        const uint32_t w = pq - slot * tile_px;
                        if (blocked8) {
                            const uint32_t b = w >> 6, l = w & 63, bpr = (uint32_t)P->tile_w >> 3;
                            const uint32_t by = udiv(b, P->u_bpr);
                            x = (b - by * bpr) * 8 + (l & 7);
                            y = by * 8 + (l >> 3);
                        } else {
                            y = udiv(w, P->u_tw);
                            x = w - y * (uint32_t)P->tile_w;
                        }
                    }
                    const uint32_t item = slot * tile_px + y * (uint32_t)P->tile_w + x;
                    const uint32_t pos = (uint32_t)P->rank + slot * (uint32_t)P->world_size;
                    const uint32_t tile = P->order ? (uint32_t)P->order[pos] : pos;  // -1: empty slot
                    const uint32_t ty = udiv(tile, P->u_tx), tx = tile - ty * (uint32_t)P->tiles_x;
                    const uint32_t pi = tile == 0xFFFFFFFFu ? 0xFFFFFFFFu : tx * (uint32_t)P->tile_w + x;
                    const uint32_t pj = tile == 0xFFFFFFFFu ? 0xFFFFFFFFu : ty * (uint32_t)P->tile_h + y;
                    if (pi >= (uint32_t)cam.image_width || pj >= (uint32_t)cam.image_height) {
                        if (!kFixed && !P->chunk && !P->direct) {  // padding pixel (chunked: gs_combine_kernel writes it)
                            if (P->out) {
                                float* o = P->out + (size_t)item * 3;
                                o[0] = 0.0f;
                                o[1] = 0.0f;
                                o[2] = 0.0f;
                            }
                            if (P->out8) {
                                uint8_t* o8 = P->out8 + (size_t)item * 3;
                                o8[0] = 0;
                                o8[1] = 0;
                                o8[2] = 0;
                            }
                        }
                    } else {
                        LI(L_PIX) = pj * (uint32_t)cam.image_width + pi;
                        LD(L_CSR) = 0.0;
                        LD(L_CSG) = 0.0;
                        LD(L_CSB) = 0.0;
                        if (kRsplit || (!kFixed && P->per_sample)) {
                            // batch rounds: the sample slots of entry pr, samples ck * csz on
                            LI(L_ITEM) = GS_ROUND_PIXEL_MAJOR ? pr * P->ss.batch_size + ck * csz : ck * csz * P->seg_n + pr;
                            LI(L_SAMPLE) = P->round_base + ck * csz;
                            LI(L_BLEFT) = min(csz, P->ss.batch_size - ck * csz);
                        } else if (kFixed || P->chunk) {
                            // chunk sums, chunk-major: a coarse pixel's at ck * fine_px + item,
                            // a fine one's after every coarse pixel's (the packed pixel and its
                            // queue position share a tile, so both are in the fine region or neither)
                            LI(L_ITEM) = fine ? P->fine_base + ck * (P->capacity - P->fine_px) + (item - P->fine_px)
                                              : ck * P->fine_px + item;
                            LI(L_SAMPLE) = ck * csz;
                            LI(L_BLEFT) = min(csz, P->ss.batch_size - ck * csz);
                            if (ck == 0) atomicAdd(&s_cnt[C_PIX], 1ull);
                        } else if (P->rounds) {
                            // batch rounds, whole-batch items: the pixel's running sums (none
                            // before round 1), then batch `round` in this lane
                            if (P->round_base) {
                                const double* ps = P->pstate + (size_t)item * 5;
                                LD(L_CSR) = ps[0];
                                LD(L_CSG) = ps[1];
                                LD(L_CSB) = ps[2];
                                LD(L_LSUM) = ps[3];
                                LD(L_LSQ) = ps[4];
                            } else {
                                LD(L_LSUM) = 0.0;
                                LD(L_LSQ) = 0.0;
                            }
                            // sample_count after this batch: 0.0 + bs + ... (exact integers)
                            LD(L_SCOUNT) = (double)((uint64_t)P->round_base + P->ss.batch_size);
                            LI(L_ITEM) = item;
                            LI(L_BLEFT) = P->ss.batch_size;
                            LI(L_SAMPLE) = P->round_base;
                        } else {
                            LD(L_LSUM) = 0.0;
                            LD(L_LSQ) = 0.0;
                            // first batch starts (camera.rs:137)
                            LD(L_SCOUNT) = 0.0 + (double)P->ss.batch_size;
                            LI(L_ITEM) = item;
                            LI(L_BLEFT) = P->ss.batch_size;
                            LI(L_SAMPLE) = 0u;
                        }
                        st = S_CAM;
                    }
                }
            }
            need = __builtin_amdgcn_ballot_w64(st == S_NEED);
        }
        // Camera rays in batches (round 5): get_ray's draws, the defocus rejection loop and
        // the stream seed cost a wave as much for a few lanes as for all 64, and after a
        // shade pass only the lanes whose sample ended (~20 of 57 on C4) want one.  So a
        // wave waits until `cam_batch` lanes want a camera ray -- those lanes sit idle, like
        // finished lanes, meanwhile -- unless no lane has a ray to trace or the queue is
        // done.  Each lane's samples and draws are unchanged; only when they start moves.
        const uint64_t cam_m = __builtin_amdgcn_ballot_w64(st == S_CAM);
        if (cam_m != 0 && ((uint32_t)__popcll(cam_m) >= (uint32_t)A.cam_batch || qdone ||
                           __builtin_amdgcn_ballot_w64(st == S_TRACE) == 0)) {
#ifdef GS_STAMPS
            it_adv++;
            ln_adv += (uint64_t)__popcll(cam_m);
#endif
            if (st == S_CAM) {
                GS_MARK("adv_begin");
                advance();
                GS_MARK("adv_end");
            }
        }
        if (qdone || __builtin_amdgcn_ballot_w64(st == S_NEED) == 0) break;
        }
        if (fresh) {  // scattered rays (shade pass) and camera rays together
            begin_ray();
            fresh = false;
        }
        if (st == S_NEED) st = S_DONE;
        if (__builtin_amdgcn_ballot_w64(st == S_TRACE || st == S_SHADE) == 0) break;
        GS_STAMP(ts1);

        // ------------------------------------------------------- traverse
        // Within this phase a lane is TRACE, SHADE or DONE and rays do not change, so the
        // shade count and the slab flavour are wave-uniform SGPR facts: no per-iteration
        // ballot for the former, a scalar branch (no exec-mask juggling) for the latter.
        const uint64_t alive = __builtin_amdgcn_ballot_w64(st != S_DONE);
        // (GS_FEAT_NESTED: a lane's ray changes when it enters or leaves a BVH under an
        // instance, in a leaf pass: recomputed there)
        bool wave_fast = __builtin_amdgcn_ballot_w64(st == S_TRACE && !fast) == 0;
        // Invariant: cur != THR_END exactly for lanes whose ray is still being traced
        // (every other lane holds THR_END), so the loop reads lane states from `cur` alone
        // and only marks finished lanes S_SHADE once it ends.
#ifdef GS_WATCHDOG
        uint32_t wd_trav = 0;
#endif
#pragma unroll 1
        for (;;) {
#ifdef GS_WATCHDOG
            if (++wd_trav > (uint32_t)GS_WATCHDOG) {
                wd_trip("traverse", wd_trav);
                break;
            }
#endif
            const uint64_t tr = __builtin_amdgcn_ballot_w64(cur != THR_END);
            if (tr == 0) break;
            if ((uint32_t)__popcll(alive & ~tr) >= (uint32_t)A.shade_batch) break;
            // Leaf batching: step nodes until `leaf_batch` tracing lanes sit at a leaf (or all
            // do), then test those leaves together, so a wave pays for the node step and the
            // sphere test in different iterations instead of both in every one.  Each lane
            // still processes its refs in the reference's order.  The pass kind is uniform.
            const bool at_leaf = cur > THR_END;
            const uint64_t lm = __builtin_amdgcn_ballot_w64(at_leaf);
            const bool leaf_pass = lm == tr || (uint32_t)__popcll(lm) >= (uint32_t)A.leaf_batch;
#ifdef GS_STAMPS
            uint64_t tp0;
            GS_STAMP(tp0);
            it_all++;
            it_node += !leaf_pass;
            it_leaf += leaf_pass;
            ln_node += leaf_pass ? 0ull : (uint64_t)__popcll(tr & ~lm);
            ln_leaf += leaf_pass ? (uint64_t)__popcll(lm) : 0ull;
#endif
            if (!leaf_pass) {
                GS_MARK("node_begin"); GS_PRIO_SET(GS_PRIO_NODE);
// A node pass takes up to GS_NODE_STEPS node steps per lane, unrolled (the loop head's
// ballots, shade-count and pass-kind tests are paid once per pass, not per node):
// measured on MI355X C4 (leaf batch 12), Msamples/s: 1 step 5487, 2 5788, 4 6049, 8 6205;
// unrolled 4 6303, 6 6384, 8 6451-6456, 10 6417, 12 6334, 16 6378; a ballot to leave the
// pass early once no lane is at a node cost 6% (8 steps: 5833).
#ifndef GS_NODE_STEPS
#define GS_NODE_STEPS 8
#endif
                // FAST (compile time): the wave's rays are all cert rays (wave_fast, uniform
                // for the pass), so the 8 unrolled steps carry no per-step flavour test.
                // LDSP (compile time): no node lane of the wave sits at a record outside the
                // LDS mirror when the pass starts (always with the whole tree mirrored), so a
                // step's one compare, cur < lim, picks the lanes that step -- and reads LDS; a
                // lane whose walk leaves the mirror parks there until the next pass, which
                // then runs the mixed flavour (each step splitting its lanes by memory).
                const uint32_t lim = (FEAT & GS_FEAT_LDSTREE) != 0 ? (uint32_t)THR_END : A.lds_nodes << 5;
                auto node_step = [&](auto fast_tag, auto ldsp_tag) __attribute__((always_inline)) {
                constexpr bool FAST = decltype(fast_tag)::value;
                constexpr bool LDSP = decltype(ldsp_tag)::value;
#ifdef GS_STAMPS
                {
                    const bool glob = !((FEAT & GS_FEAT_LDSTREE) != 0) && cur < THR_END && cur >= (A.lds_nodes << 5);
                    const uint64_t act = __builtin_amdgcn_ballot_w64(LDSP ? cur < lim : cur < THR_END);
                    const uint64_t gl = __builtin_amdgcn_ballot_w64(glob && !LDSP);
                    d_gvis += glob && !LDSP;
                    d_wsteps += act != 0;
                    d_wsteps_g += gl != 0;
                    d_wlanes += (uint64_t)__popcll(act);
                }
#endif
                if (__builtin_expect(LDSP ? cur < lim : cur < THR_END, 1)) {
                    // One 32-B record (2 x 16 B; from LDS, offset = cur, or off the SGPR
                    // base), the box test, and the next record: the hit link or the miss link.
                    u32x4 ra, rb;
                    if constexpr (LDSP) {
                        ra = *(lds_u32x4*)(uintptr_t)cur;
                        rb = *(lds_u32x4*)(uintptr_t)node_half_b(cur);
                    } else {
                        load_tnode_w<(FEAT & GS_FEAT_LDSTREE) != 0>(s_nodes, A.tnodes, cur, A.lds_nodes << 5, ra, rb);
                    }
                    c_nodes++;
                    if constexpr ((FEAT & GS_FEAT_VISITS) != 0) {
                        if (P->visits) count_visit(P->visits, cur >> 5);
                    }
                    const uint32_t me = cur;  // this record
                    if constexpr (FAST) {
                        // the certified decision picks the link at once; lanes f32 cannot
                        // decide (rare) run the reference's f64 test out of line.  (Taking the
                        // link once after the join saves the copy of `cur` but puts the hit
                        // mask in an SGPR pair: VOP3 compare and select, +2 issue cycles.)
                        float d, thr;
                        bool h = box_cert_dt(__uint_as_float(ra.x), __uint_as_float(ra.y), __uint_as_float(rb.x),
                                             __uint_as_float(ra.z), __uint_as_float(ra.w), __uint_as_float(rb.y), rc,
                                             tmin32, closest32, d, thr);
                        cur = h ? rb.z : rb.w;
                        if (__builtin_expect(__builtin_fabsf(d) <= thr, 0)) {  // undecided by f32: the f64 test
                            GS_MARK("fallback_begin");
                            h = box_hit_fast(box64(A.tboxes[me >> 5]), ray.o, inv_of(ray.d), tmin, closest);
                            cur = h ? rb.z : rb.w;
                            GS_MARK("fallback_end");
                        }
#ifdef GS_CERT_CHECK
                        // Diagnostic build: every certified decision re-checked in f64; a
                        // mismatch is counted (counters[15]) and its first 64 cases recorded
                        // (item_visits as f64[64][16]: o, d, f64 box, tmin, closest, f32 verdict).
                        {
                            const TBox bx = A.tboxes[me >> 5];
                            const bool h64 = box_hit(box64(bx), ray.o, inv_of(ray.d), tmin, closest);
                            if (h64 != h) {
                                const unsigned long long k = atomicAdd(&P->counters[15], 1ull);
                                if (k < 64 && P->item_visits) {
                                    double* rec = reinterpret_cast<double*>(P->item_visits) + k * 16;
                                    const double v[16] = {ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z, bx.mnx,
                                                          bx.mny, bx.mnz, bx.mxx, bx.mxy, bx.mxz, tmin, closest,
                                                          (double)h, (double)closest32};
                                    for (int q = 0; q < 16; q++) rec[q] = v[q];
                                }
                            }
                        }
#endif
                    } else {  // a wave with a non-cert ray: the f64 compare-select test
                        GS_MARK("slow_begin");
                        const bool h = box_hit(box64(A.tboxes[me >> 5]), ray.o, inv_of(ray.d), tmin, closest);
                        cur = h ? rb.z : rb.w;
                        GS_MARK("slow_end");
                    }
                }
                };
                // The scene's step count (gs_device_scene.node_steps): the full count as one
                // unrolled block (a runtime exit inside it keeps the loop rolled: -1.5% on C4),
                // fewer steps (trees of other-kind leaves) as a loop.  The mixed-memory flavour
                // (a node lane outside the mirror at the pass start: ~10% of C4's passes) and
                // waves holding a non-cert ray (rare) take rolled loops.
                using fast_t = std::integral_constant<bool, true>;
                using slow_t = std::integral_constant<bool, false>;
                using ldsp_t = std::integral_constant<bool, true>;
                using mixed_t = std::integral_constant<bool, false>;
                const bool lds_pass = (FEAT & GS_FEAT_LDSTREE) != 0 ||
                                      __builtin_amdgcn_ballot_w64(cur < THR_END && cur >= lim) == 0;
                if (wave_fast && lds_pass && A.node_steps >= kUnroll) {
#pragma unroll
                    for (int nstep = 0; nstep < kUnroll; nstep++) node_step(fast_t{}, ldsp_t{});
                } else if (wave_fast && lds_pass && A.node_steps == 1) {  // (trees of other-kind leaves, C3)
                    node_step(fast_t{}, ldsp_t{});
                } else if (wave_fast && lds_pass) {
#pragma unroll 1
                    for (int nstep = 0; nstep < A.node_steps; nstep++) node_step(fast_t{}, ldsp_t{});
                } else if (wave_fast) {
#pragma unroll 1
                    for (int nstep = 0; nstep < A.node_steps; nstep++) node_step(fast_t{}, mixed_t{});
                } else {
#pragma unroll 1
                    for (int nstep = 0; nstep < A.node_steps; nstep++) node_step(slow_t{}, mixed_t{});
                }
                GS_MARK("node_end"); GS_PRIO_CLR(GS_PRIO_NODE);
            } else if (kNested && __builtin_amdgcn_ballot_w64(cur == THR_RET) != 0) {
                // Return passes (GS_FEAT_NESTED): a lane whose walk of a BVH under an instance
                // chain ended (the tree's last links are THR_RET) takes back its top-level ray
                // and goes on at the record after the instance's leaf -- where BVHNode::hit's
                // recursion returns from the Translate / RotateY's hit (hittable.rs:107-211).
#ifdef GS_STAMPS
                uint64_t rt0_;
                GS_STAMP(rt0_);
#endif
                if (cur == THR_RET) {
                    ray.o = mk(NSAVE(0), NSAVE(1), NSAVE(2));
                    ray.d = mk(NSAVE(3), NSAVE(4), NSAVE(5));
                    cur = (uint32_t)__double_as_longlong(NSAVE(6));
                    LNINST = GS_REF_NONE;
                }
                GS_REGION(6, rt0_);  // (stamps: return passes)
            } else if (at_leaf) {
                GS_MARK("leaf_begin"); GS_PRIO_SET(GS_PRIO_LEAF);
                double scx, scy, scz, sr;
                uint32_t next, ref;
                load_tleaf<(FEAT & GS_FEAT_LDSTREE) != 0>(s_leaves, A.tleaves, cur & ~THR_LEAF, A.lds_leaves, scx, scy, scz, sr,
                                                         next, ref);
                // Kind-batched leaf passes (GS_LEAF_KIND_BATCH): besides stationary spheres, a
                // pass tests only the leaves of one other kind (the first such lane's); lanes
                // at other kinds keep their leaf for a later pass, so each kind's code runs
                // with its lanes together instead of every kind present running in turn.  On
                // for kernels with BVHs under instances or staged shading, where many kinds
                // meet: final_scene +8.5%, C5 +1.3%; off elsewhere (C3 -1.2%, cornell_smoke
                // -0.4%; profiles/r03/ab_leaf_kind_batch.txt).  Each lane still tests its own
                // leaves in its own order, so nothing it computes changes.
#ifndef GS_LEAF_KIND_BATCH
#define GS_LEAF_KIND_BATCH ((FEAT & (GS_FEAT_NESTED | GS_FEAT_MIXED)) != 0)
#endif
                bool take_leaf = true;
                if constexpr (GS_LEAF_KIND_BATCH && (FEAT & GS_FEAT_SPHLEAF) == 0) {
                    const uint32_t kind = ref >> GS_REF_SHIFT;
                    const uint64_t om = __builtin_amdgcn_ballot_w64(kind != GS_REF_SPHERE);
                    if (om != 0) {
                        const uint32_t k0 = __builtin_amdgcn_readlane(kind, (uint32_t)__builtin_ctzll(om));
                        take_leaf = kind == GS_REF_SPHERE || kind == k0;
                    }
                }
                if (take_leaf) {
                if constexpr ((FEAT & GS_FEAT_VISITS) != 0) {
                    if (P->visits) count_visit(P->visits, P->visit_leaf_base + (cur & ~THR_LEAF));
                }
#ifdef GS_STAMPS
                {  // counted by the pass's first active lane (summed over lanes at the end)
                    // The r03 hang of this build on media scenes was in these counts: its
                    // distinct-KIND loop took `readlane(ref, L) >> GS_REF_SHIFT`, and the builtin
                    // returns int, so the scalar shift was arithmetic while each lane's
                    // `ref >> GS_REF_SHIFT` was logical: a medium's ref (kind 8, bit 31) never
                    // matched its own lane and the mask never emptied (ISA:
                    // profiles/r05/ballot_anomaly_isa.txt).  The readlane results are uint32_t
                    // here, the kinds come from the ref loop, and the picked lane is retired
                    // whatever the ballot returns; dbg[23] counts passes whose ballot missed it.
                    const uint64_t act = __builtin_amdgcn_read_exec();
                    const bool first = __builtin_ctzll(act) == (uint32_t)lane;
                    bool bad = false;
                    uint32_t kinds = 0;
                    uint64_t m = act;
                    while (m) {
                        const uint32_t L = (uint32_t)__builtin_ctzll(m);
                        const uint32_t r0 = __builtin_amdgcn_readlane(ref, L);
                        const uint64_t same = __builtin_amdgcn_ballot_w64(ref == r0);
                        bad |= ((same >> L) & 1u) == 0;
                        kinds |= 1u << (r0 >> GS_REF_SHIFT);
                        m &= ~(same | (1ull << L));
                        dist_ref += first;
                    }
                    dist_kind += first ? (uint64_t)__builtin_popcount(kinds) : 0;
                    dist_bad += bad && first;
                }
#endif
                // a stationary sphere's test (sphere.rs:64-106); its root divisions through one
                // refined reciprocal of a when every active lane's a is in range (as the
                // sphere-only leaf runs below), else the f64 division
                auto sphere_test = [&](d3 c, double rr, double& t) __attribute__((always_inline)) {
                    const double a = len2(ray.d);
                    // (not in media / nested-BVH kernels: final_scene and cornell_smoke measured
                    // neutral, and the media kernel spilled 12 B/lane with it)
                    constexpr bool kRa = GS_ROOT_RCP && (FEAT & (GS_FEAT_MEDIA | GS_FEAT_NESTED)) == 0;
                    if (kRa && __builtin_amdgcn_ballot_w64(!(a >= 0x1p-900 && a <= 0x1p900)) == 0)
                        return sphere_accept_rr_ra(c, rr, ray, a, rcp_cert(a), tmin, closest, t);
                    return sphere_accept_rr(c, rr, ray, a, tmin, closest, t);
                };
                auto sphere_leaf = [&]() __attribute__((always_inline)) {  // a stationary sphere, inline
                    GS_MARK("sphere_begin");
                    count_sph();
                    double t;
                    if (sphere_test(mk(scx, scy, scz), sr, t)) {
                        closest = t;
                        closest32 = (float)t;
                        hit_ref = ref;
                        if constexpr (kNested) LI(L_HINST) = LNINST;  // (a sphere of the tree under LNINST)
                        else if constexpr (!kSphLeaf) LI(L_HINST) = GS_REF_NONE;
                    }
                    GS_MARK("sphere_end");
                };
                if constexpr ((FEAT & GS_FEAT_SPHLEAF) != 0) {
                    // Sphere-only trees: a leaf run's second sphere (the next record, when it
                    // is a leaf) is read right away and both discriminants are computed as two
                    // independent chains; the roots are then taken in order, the second sphere
                    // against the interval the first left (sphere.rs:64-89, BVH.rs:73-80).
                    const bool two = cur_next_is_leaf(next);
                    double s2x, s2y, s2z, s2r;
                    uint32_t next2, ref2;
                    load_tleaf<(FEAT & GS_FEAT_LDSTREE) != 0>(s_leaves, A.tleaves, two ? next & ~THR_LEAF : cur & ~THR_LEAF,
                                                             A.lds_leaves, s2x, s2y, s2z, s2r, next2, ref2);
                    const double a = len2(ray.d);
                    // Root rounds (round 5): the square root and the divisions run once for
                    // the lane's first sphere with a real discriminant (sphere 1, else sphere 2),
                    // then once more only for lanes where both were real.  Run per sphere, both
                    // root blocks executed in most passes (C4 traces: 86% and 76% of leaf passes;
                    // in rounds 97% and 19%).  MI355X C4: 8 025 -> 8 226 Msamples/s.  Order: a
                    // lane whose sphere 1 is real takes it against `closest`, then sphere 2
                    // against what it left; a lane whose sphere 1 is not real takes sphere 2
                    // first, as the reference, whose sphere-1 test changed nothing.
                    const SphereDisc q1 = sphere_disc_rr(mk(scx, scy, scz), sr, ray, a);
                    const SphereDisc q2 = sphere_disc_rr(mk(s2x, s2y, s2z), s2r, ray, a);
                    const bool real1 = !(q1.disc < 0.0), real2 = two && !(q2.disc < 0.0);
                    GS_MARK("sphere_begin");
                    double t;
                    // Root divisions by a from one refined reciprocal per pass (sphere_root_take_ra,
                    // bit-identical for a in [2^-900, 2^900]: a wave-uniform choice, else `/`)
                    const double ra = rcp_cert(a);
                    const bool wave_ra =
                        GS_ROOT_RCP && __builtin_amdgcn_ballot_w64(!(a >= 0x1p-900 && a <= 0x1p900)) == 0;
                    auto take = [&](double hh, double dd) __attribute__((always_inline)) {
                        return wave_ra ? sphere_root_take_ra(hh, dd, a, ra, tmin, closest, t)
                                       : sphere_root_take(hh, dd, a, tmin, closest, t);
                    };
                    if (real1 || real2) {
                        const double hA = real1 ? q1.h : q2.h, dA = real1 ? q1.disc : q2.disc;
                        if (take(hA, dA)) {
                            closest = t;
                            hit_ref = real1 ? ref : ref2;
                        }
                    }
                    if (real1 && real2) {
                        if (take(q2.h, q2.disc)) {
                            closest = t;
                            hit_ref = ref2;
                        }
                    }
                    if (two) {
                        if constexpr ((FEAT & GS_FEAT_VISITS) != 0) {
                            if (P->visits) count_visit(P->visits, P->visit_leaf_base + (next & ~THR_LEAF));
                        }
                        next = next2;
                    }
                    closest32 = (float)closest;
                    c_sph += 1u + (uint32_t)two;
                    GS_MARK("sphere_end");
                } else if ((FEAT & GS_FEAT_SPHLEAF) != 0 || (ref >> GS_REF_SHIFT) == GS_REF_SPHERE) {
#ifdef GS_STAMPS
                    uint64_t k0_;
                    GS_STAMP(k0_);
#endif
                    sphere_leaf();
                    GS_REGION(7 + GS_REF_SPHERE, k0_);
                } else if constexpr ((FEAT & GS_FEAT_SPHLEAF) == 0) {
                    GS_MARK("other_begin");
#ifdef GS_STAMPS
                    // (leaf-kind clock: the branch's first lane's ref kind, before any
                    // instance chain -- one kind per pass with kind-batched leaf passes)
                    uint64_t k0_;
                    GS_STAMP(k0_);
                    const uint32_t kk_ = __builtin_amdgcn_readfirstlane(ref >> GS_REF_SHIFT);
#endif
                    // A leaf pass whose other-kind lanes all sit at one leaf (the Cornell box:
                    // always, with single node steps) tests it with scalar loads.
                    const uint32_t r0 = __builtin_amdgcn_readfirstlane(ref);
                    const bool uni = __builtin_amdgcn_ballot_w64(ref != r0) == 0;
                    LeafHit lh;
                    Ray rl = ray;  // (the ray in the leaf's space after its instance chain)
                    if (uni) lh = leaf_other<FEAT, true>(sc, qs, r0, rl, tmin, closest, rng, s_cnt);
                    else lh = leaf_other<FEAT, false>(sc, qs, ref, rl, tmin, closest, rng, s_cnt);
                    if (lh.hit) {
                        closest = lh.t;
                        closest32 = (float)lh.t;
                        hit_ref = lh.ref;
                        // (a primitive or list in the tree under LNINST; an instance leaf's own chain;
                        // round 6: an instance leaf inside the tree under LNINST -- both chains, the
                        // outer one in the save slot, bit 31 on the inner one)
                        if constexpr (kNested && kGeneral) {
                            if (lh.inst != GS_REF_NONE && LNINST != GS_REF_NONE) {
                                NSAVE(7) = __longlong_as_double((long long)LNINST);
                                LI(L_HINST) = lh.inst | 0x80000000u;
                            } else {
                                LI(L_HINST) = lh.inst != GS_REF_NONE ? lh.inst : LNINST;
                            }
                        } else if constexpr (kNested) {
                            LI(L_HINST) = lh.inst != GS_REF_NONE ? lh.inst : LNINST;
                        } else {
                            LI(L_HINST) = lh.inst;
                        }
                    }
                    if constexpr (kNested) {
                        // The chain ended in a BVH (final_scene's box of balls): the lane walks
                        // the tree in the main loop's node and leaf passes, in the reference's
                        // order, with its ray in the tree's space; the top-level ray and the
                        // link after this leaf wait in the lane's save slot until THR_RET.
                        if (lh.enter) {
                            NSAVE(0) = ray.o.x;
                            NSAVE(1) = ray.o.y;
                            NSAVE(2) = ray.o.z;
                            NSAVE(3) = ray.d.x;
                            NSAVE(4) = ray.d.y;
                            NSAVE(5) = ray.d.z;
                            NSAVE(6) = __longlong_as_double((long long)next);
                            LNINST = ref;
                            ray.o = rl.o;
                            ray.d = rl.d;
                            next = sc.nroots[lh.enter - 1u];
                        }
                    }
                    GS_REGION(7 + (kk_ < 1u ? 1u : kk_ > 8u ? 8u : kk_), k0_);
                    GS_MARK("other_end");
                }
                cur = next;
#ifndef GS_LEAF_RUN
#define GS_LEAF_RUN 2
#endif
                // More leaves in the same pass while the next record is a leaf holding a
                // stationary sphere (the n == 2 leaves of BVH.rs:44-55 sit side by side):
                // up to GS_LEAF_RUN per pass, each tested in order with the updated closest.
                // A template feature: trees without such pairs (the Cornell box's quads and
                // instances) lose ~2% to the loop's mere presence (MI355X C3).
#pragma unroll 1
                for (int k = 1; (FEAT & GS_FEAT_LEAFRUN) && (FEAT & GS_FEAT_SPHLEAF) == 0 &&
                                k < GS_LEAF_RUN && cur > THR_END && (!kNested || cur != THR_RET); k++) {
                    load_tleaf<(FEAT & GS_FEAT_LDSTREE) != 0>(s_leaves, A.tleaves, cur & ~THR_LEAF, A.lds_leaves, scx, scy, scz, sr,
                                                         next, ref);
                    if ((FEAT & GS_FEAT_SPHLEAF) == 0 && (ref >> GS_REF_SHIFT) != GS_REF_SPHERE) break;
                    if constexpr ((FEAT & GS_FEAT_VISITS) != 0) {
                        if (P->visits) count_visit(P->visits, P->visit_leaf_base + (cur & ~THR_LEAF));
                    }
                    count_sph();
                    double t;
                    if (sphere_test(mk(scx, scy, scz), sr, t)) {
                        closest = t;
                        closest32 = (float)t;
                        hit_ref = ref;
                        if constexpr (kNested) LI(L_HINST) = LNINST;
                        else if constexpr (!kSphLeaf) LI(L_HINST) = GS_REF_NONE;
                    }
                    cur = next;
                }
                }  // take_leaf
                GS_MARK("leaf_end"); GS_PRIO_CLR(GS_PRIO_LEAF);
            }
            // Nested-BVH kernels and media kernels with sphere leaf runs: the certified test's
            // ray constants are recomputed after a leaf pass (the same function of the same
            // ray), so they are not live through leaf_other, whose medium and nested tests
            // need the registers (without it these spill 12-36 B/lane).  Media-only kernels
            // (cornell_smoke: a leaf pass after nearly every single node step) have the
            // registers and skip the recomputation (with it: -6.6%).
            // In nested-BVH kernels a lane's ray also changes in a leaf pass (entering or leaving a
            // BVH under an instance): its slab flavour is decided again, and the wave's.
            if constexpr ((FEAT & GS_FEAT_NESTED) != 0 ||
                          (FEAT & (GS_FEAT_MEDIA | GS_FEAT_LEAFRUN)) == (GS_FEAT_MEDIA | GS_FEAT_LEAFRUN)) {
                if (leaf_pass) {
#ifdef GS_STAMPS
                    uint64_t rc0_;
                    GS_STAMP(rc0_);
#endif
                    const d3 inv = inv_cert(ray.d);
                    rc = make_cert(ray.o, inv);
                    if constexpr (kNested) {
                        fast = A.cert_boxes && cert_ray_ok(ray.o, inv);
                        wave_fast = __builtin_amdgcn_ballot_w64(cur != THR_END && !fast) == 0;
                    }
                    GS_REGION(5, rc0_);  // (stamps: the recomputation's share of the leaf-pass clock)
                }
            }
#ifdef GS_STAMPS
            {
                uint64_t tp1;
                GS_STAMP(tp1);
                (leaf_pass ? acc_leaf : acc_node) += tp1 - tp0;
            }
#endif
        }
        if (st == S_TRACE && cur == THR_END) st = S_SHADE;

        // ---------------------------------------------------------- shade
        GS_STAMP(ts2);
#ifdef GS_STAMPS
        {
            const uint64_t sm = __builtin_amdgcn_ballot_w64(st == S_SHADE);
            it_shade += sm != 0;
            ln_shade += (uint64_t)__popcll(sm);
        }
#endif
        if (st == S_SHADE) {
            bool ends = true;
            double Lr = 0.0, Lg = 0.0, Lb = 0.0;
#ifdef GS_STAMPS
            uint64_t r0;
#endif
            if constexpr ((FEAT & (GS_FEAT_MIXED | GS_FEAT_MEDIA | GS_FEAT_NESTED)) != 0) {
                GS_STAMP(r0);
                GS_MARK("shade_begin"); GS_PRIO_SET(GS_PRIO_SHADE);
#if defined(GS_DIAG_DUP) && (GS_DIAG_DUP & 1)
                {  // cost probe: the shade work twice (the copy's results consumed, its counts double)
                    Ray r2 = ray;
                    uint64_t g2 = rng;
                    double c2 = closest;
                    asm volatile("" : "+v"(r2.d.x), "+v"(c2));
                    const ShadeOut s2 = shade<(FEAT & GS_FEAT_PLAIN) != 0, kSphLeaf, kGeneral>(sc, r2, c2, hit_ref, LI(L_HINST), g2, s_cnt);
                    asm volatile("" ::"v"(s2.col.x), "v"(s2.col.y), "v"(s2.col.z), "v"(s2.dir.x), "v"(s2.dir.y), "v"(s2.dir.z),
                                 "v"(r2.o.x), "v"(g2), "v"(s2.cont));
                }
#endif
                // (GS_FEAT_NESTED: a hit through a chain inside a BVH under another chain carries
                // bit 31 on its inner chain's ref, the outer chain in the lane's save slot 7)
                uint32_t hinst = (FEAT & GS_FEAT_PLAIN) ? GS_REF_NONE : LI(L_HINST), houter = GS_REF_NONE;
                if constexpr (kNested && kGeneral) {
                    if (hinst != GS_REF_NONE && (hinst >> 31)) {
                        houter = (uint32_t)__double_as_longlong(NSAVE(7));
                        hinst &= 0x7FFFFFFFu;
                    }
                }
                const ShadeOut s = shade<(FEAT & GS_FEAT_PLAIN) != 0, kSphLeaf, kGeneral>(sc, ray, closest, hit_ref, hinst,
                                                                                        rng, s_cnt, houter);
                GS_MARK("shade_end"); GS_PRIO_CLR(GS_PRIO_SHADE);
                GS_REGION(2, r0);
                if (s.cont) {
                    Tr = Tr * s.col.x;
                    Tg = Tg * s.col.y;
                    Tb = Tb * s.col.z;
                    const uint32_t depth = LI(L_DEPTH) - 1u;
                    LI(L_DEPTH) = depth;
                    if (depth > 0) {
                        ray.d = s.dir;  // (ray.o = p: set by shade)
                        fresh = true;
                        st = S_TRACE;
                        ends = false;
                    }  // else ray_color(.., 0) = 0 (camera.rs:175): black
                } else {
                    // sky (camera.rs:201), emitter (DiffuseLight never scatters) or absorbed (col = 0)
                    Lr = Tr * s.col.x;
                    Lg = Tg * s.col.y;
                    Lb = Tb * s.col.z;
                }
            } else {  // split: one branch per case
                if (hit_ref == GS_REF_NONE) {
                    // miss: sample_background (camera.rs:201); the path's only radiance
                    GS_STAMP(r0);
                    const d3 bg = background(sc, ray.d, s_cnt);
                    GS_REGION(0, r0);
                    Lr = Tr * bg.x;
                    Lg = Tg * bg.y;
                    Lb = Tb * bg.z;
                } else {
                    atomicAdd(&s_cnt[C_HITS], 1ull);
                    GS_STAMP(r0);
                    const HitRec h = kSphLeaf ? reconstruct_sphere<true>(sc, ray, closest, hit_ref)
                                              : reconstruct<false>(sc, ray, closest, hit_ref, LI(L_HINST));
                    GS_REGION(1, r0);
                    GS_STAMP(r0);
                    const Scatter s = scatter(sc, h, ray.d, rng, s_cnt);
                    GS_REGION(2, r0);
                    rng = s.rng;
                    if (s.cont) {
                        Tr = Tr * s.col.x;
                        Tg = Tg * s.col.y;
                        Tb = Tb * s.col.z;
                        const uint32_t depth = LI(L_DEPTH) - 1u;
                        LI(L_DEPTH) = depth;
                        if (depth > 0) {
                            ray.o = h.p;
                            ray.d = s.dir;
                            fresh = true;
                            st = S_TRACE;
                            ends = false;
                        }  // else ray_color(.., 0) = 0 (camera.rs:175): black
                    } else {
                        // emitter (DiffuseLight never scatters) or absorbed (col = 0)
                        Lr = Tr * s.col.x;
                        Lg = Tg * s.col.y;
                        Lb = Tb * s.col.z;
                    }
                }
            }
            if (ends) {  // the sample is done; its item's next camera ray comes at the loop head
                GS_STAMP(r0);
                add_sample(Lr, Lg, Lb);
                if ((kFixed || P->chunk) && LI(L_BLEFT) == 0) end_chunk();  // -> S_NEED
                else st = S_CAM;
                GS_REGION(4, r0);
            }
        }
#ifdef GS_STAMPS
        GS_STAMP(ts3);
        acc_refill += ts1 - ts0;
        acc_trav += ts2 - ts1;
        acc_shade += ts3 - ts2;
#endif
    }
#ifdef GS_STAMPS
    if (P->item_visits && (dist_ref || dist_kind || dist_bad)) {
        unsigned long long* dbg = (unsigned long long*)P->item_visits;
        atomicAdd(&dbg[17], (unsigned long long)dist_ref);
        atomicAdd(&dbg[18], (unsigned long long)dist_kind);
        atomicAdd(&dbg[23], (unsigned long long)dist_bad);
    }
    if (P->item_visits && d_gvis) atomicAdd(&((unsigned long long*)P->item_visits)[19], (unsigned long long)d_gvis);
    if (lane == 0 && P->item_visits) {
        unsigned long long* dbg = (unsigned long long*)P->item_visits;
        atomicAdd(&dbg[0], (unsigned long long)acc_refill);
        atomicAdd(&dbg[1], (unsigned long long)acc_trav);
        atomicAdd(&dbg[2], (unsigned long long)acc_shade);
        atomicAdd(&dbg[3], (unsigned long long)it_all);
        atomicAdd(&dbg[4], (unsigned long long)it_node);
        atomicAdd(&dbg[5], (unsigned long long)it_leaf);
        atomicAdd(&dbg[6], (unsigned long long)ln_node);
        atomicAdd(&dbg[7], (unsigned long long)ln_leaf);
        atomicAdd(&dbg[8], (unsigned long long)it_shade);
        atomicAdd(&dbg[9], (unsigned long long)ln_shade);
        for (int k = 0; k < 5; k++) atomicAdd(&dbg[10 + k], s_reg[(tid >> 6) * 16 + k]);
        for (int k = 0; k < 8; k++) atomicAdd(&dbg[24 + k], s_reg[(tid >> 6) * 16 + 8 + k]);
        for (int k = 5; k < 7; k++) atomicAdd(&dbg[29 + k], s_reg[(tid >> 6) * 16 + k]);  // dbg[34], dbg[35]
        atomicAdd(&dbg[15], (unsigned long long)acc_node);
        atomicAdd(&dbg[16], (unsigned long long)acc_leaf);
        atomicAdd(&dbg[20], (unsigned long long)d_wsteps);
        atomicAdd(&dbg[21], (unsigned long long)d_wsteps_g);
        atomicAdd(&dbg[22], (unsigned long long)d_wlanes);
        atomicAdd(&dbg[32], (unsigned long long)it_adv);
        atomicAdd(&dbg[33], (unsigned long long)ln_adv);

    }
#endif
#undef LD
#undef LI
#undef LNINST
#undef NSAVE
#undef Tr
#undef Tg
#undef Tb
#undef GS_TP

    // flush counters: LDS -> global, one atomic per counter per block
    atomicAdd(&s_cnt[C_NODES], (unsigned long long)c_nodes);
    atomicAdd(&s_cnt[C_SPH], (unsigned long long)c_sph);
    __syncthreads();
    // (the block's first C_N lanes: wave 0, where the lane is the thread index; the test is
    // a wave-uniform mask taken at the start, so no thread-index register is kept to here)
    const uint32_t lane_end = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if (((flushers >> lane_end) & 1ull) && P->counters) atomicAdd(&P->counters[lane_end], s_cnt[lane_end]);
}

// Per-launch parameters reach device memory by a one-thread kernel on the caller's stream
// (not a pageable hipMemcpyAsync, which can block the host until earlier work drains and
// would need a host buffer that outlives the copy).
__global__ void gs_params_kernel(KParams kp, KParams* __restrict__ dst) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        *dst = kp;
        *kp.queue = 0u;  // (here rather than a memset: one stream operation fewer per frame)
    }
    if (kp.zero_counters && blockIdx.x == 0 && threadIdx.x < sizeof(gs_counters) / 8) kp.counters[threadIdx.x] = 0ull;
}

// Chunked single-batch renders: a pixel's colour is the sum of its chunks' Σrgb, taken
// in chunk (= sample) order, over the batch size (camera.rs:142-160 with one batch).
// Padding slots of partial tiles get zeros.
// Packed pixel k of this rank -> its image pixel (pi, pj); false for a padding slot (an empty
// tile slot of the plan, or outside the image).
__device__ __forceinline__ bool packed_pixel(const KParams* __restrict__ P, uint32_t k, uint32_t& pi, uint32_t& pj) {
    const uint32_t tile_px = (uint32_t)(P->tile_w * P->tile_h);
    const uint32_t slot = k / tile_px, w = k % tile_px;
    const uint32_t pos = (uint32_t)P->rank + slot * (uint32_t)P->world_size;
    const uint32_t tile = P->order ? (uint32_t)P->order[pos] : pos;  // -1: empty slot
    if (tile == 0xFFFFFFFFu) return false;
    pi = (tile % (uint32_t)P->tiles_x) * (uint32_t)P->tile_w + w % (uint32_t)P->tile_w;
    pj = (tile / (uint32_t)P->tiles_x) * (uint32_t)P->tile_h + w / (uint32_t)P->tile_w;
    return pi < (uint32_t)P->cam.image_width && pj < (uint32_t)P->cam.image_height;
}

__global__ void gs_combine_kernel(const KParams* __restrict__ P) {
    const uint32_t cpp = P->cpp;
    const double scount = 0.0 + (double)P->ss.batch_size;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < P->capacity; k += gridDim.x * blockDim.x) {
        uint32_t pi = 0, pj = 0;
        const bool real = packed_pixel(P, k, pi, pj);
        const size_t oi = P->direct ? (size_t)pj * (uint32_t)P->cam.image_width + pi : (size_t)k;
        float* o = P->out ? P->out + oi * 3 : nullptr;
        uint8_t* o8 = P->out8 ? P->out8 + oi * 3 : nullptr;
        if (!real) {
            if (P->direct) continue;
            if (o) {
                o[0] = 0.0f;
                o[1] = 0.0f;
                o[2] = 0.0f;
            }
            if (o8) {
                o8[0] = 0;
                o8[1] = 0;
                o8[2] = 0;
            }
            continue;
        }
        const bool fine = k >= P->fine_px;
        // chunk-major sums: consecutive lanes read consecutive 24-B sums of each chunk
        const size_t stride = (size_t)(fine ? P->capacity - P->fine_px : P->fine_px) * 3;
        const double* p = P->partial + (fine ? (size_t)P->fine_base + (k - P->fine_px) : (size_t)k) * 3;
        double r = 0.0, g = 0.0, b = 0.0;
        if (!fine) {
            for (uint32_t c = 0; c < cpp; c++, p += stride) {
                r += p[0];
                g += p[1];
                b += p[2];
            }
        } else {
            // 1-sample items (fine_chunk 1: each sum is 0 + s = s), re-formed into the coarse
            // chunks of P->chunk samples and added in order: the coarse pixels' association,
            // so a pixel's bits do not depend on whether its tile ran in the tail
            const uint32_t bs = P->ss.batch_size, c = P->chunk;
            for (uint32_t s0 = 0; s0 < bs; s0 += c) {
                const uint32_t e = min(bs, s0 + c);
                double cr = 0.0, cg = 0.0, cb = 0.0;
                for (uint32_t s = s0; s < e; s++, p += stride) {
                    cr += p[0];
                    cg += p[1];
                    cb += p[2];
                }
                r += cr;
                g += cg;
                b += cb;
            }
        }
        const double cr = r / scount, cg = g / scount, cb = b / scount;
        if (o) {
            o[0] = (float)cr;
            o[1] = (float)cg;
            o[2] = (float)cb;
        }
        if (o8) {
            o8[0] = color_byte(cr);
            o8[1] = color_byte(cg);
            o8[2] = color_byte(cb);
        }
    }
}

// ------------------------------------------------ adaptive sampling in batch rounds
// The reference's adaptive loop (camera.rs:135-165) runs a pixel's batches one after the
// other, each batch's stop test over the running sums.  Per-lane that puts up to
// max_samples + batch sequential samples of one pixel into one lane, and a frame ends on
// its slowest pixels (an all-black pixel never converges, camera.rs:156).  In rounds, round
// r renders batch r of every pixel still active, its samples split into work items like the
// fixed-spp chunks, each sample's colour kept; the combine then folds a pixel's batch into
// its sums in sample order and takes the stop test -- the same f64 operations in the same
// order as the sequential loop, so every stop decision and every output is bit-identical.

// Before round 0: padding slots get their zero output; every real packed pixel enters the
// first active list (one atomic per wave; the order inside a wave is kept).
__global__ void gs_round_init_kernel(const KParams* __restrict__ P) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cap = P->capacity;
    const uint32_t span = (cap + 63u) & ~63u;  // whole waves take every iteration (ballots)
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < span; k += gridDim.x * blockDim.x) {
        bool real = false;
        if (k < cap) {
            uint32_t pi = 0, pj = 0;
            real = packed_pixel(P, k, pi, pj);
            if (!real && !P->direct) {
                if (P->out) {
                    float* o = P->out + (size_t)k * 3;
                    o[0] = 0.0f;
                    o[1] = 0.0f;
                    o[2] = 0.0f;
                }
                if (P->out8) {
                    uint8_t* o8 = P->out8 + (size_t)k * 3;
                    o8[0] = 0;
                    o8[1] = 0;
                    o8[2] = 0;
                }
            }
        }
        const uint64_t m = __builtin_amdgcn_ballot_w64(real);
        if (m == 0) continue;
        const uint32_t leader = (uint32_t)__builtin_ctzll(m);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&P->round_counts[0], (uint32_t)__popcll(m));
        base = __shfl(base, (int)leader);
        if (real) P->active_buf[0][base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = k;
    }
}

// Before each (round, segment) launch: this launch's share of the round's active list, its
// chunking (finer when few pixels are left, so the round's samples still spread over the
// lanes), queue claim and cleared queue.
__global__ void gs_round_params_kernel(KParams* __restrict__ P, uint32_t round, uint32_t seg, uint32_t seg_px,
                                       int32_t chunk_req, int32_t whole_mode) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t n_act = P->round_counts[round];
    const uint32_t base = seg * seg_px;
    const uint32_t n_seg = n_act > base ? min(seg_px, n_act - base) : 0u;
    const uint32_t bs = P->ss.batch_size;
    // whole-batch items while the active pixels are at least twice the lanes (no per-sample
    // colours kept, no combine), split ones once few are left (their samples spread over the
    // lanes); a requested sample chunk always splits
    const bool whole = chunk_req <= 0 && bs <= GS_ROUND_WHOLE_MAX_BATCH &&
                       (whole_mode > 0 || (whole_mode < 0 && (uint64_t)n_seg >= 2ull * P->lanes));
    uint32_t csz;
    if (chunk_req > 0) {
        csz = min((uint32_t)chunk_req, bs);
    } else {
        // Scenes whose paths are long (>= 2 rays a path so far: the launch's counters from round
        // 1 on, before that the slot's last rounds) take 1-sample items: a round then ends on one
        // path, not on an item of several.  Round 6, MI355X A2 (cornell_box, 5.3 rays a path):
        // the rule below for every scene 9 553 Msamples/s; 16 / 32 / 64 / 128 items per lane
        // 10 216 / 10 767 / 10 955 / 10 954, the last two 1-sample items at A2's size.  Short
        // paths (A1's hdri, 1.1) keep the rule -- halve 16-sample items until the round has 8
        // items per lane: with 1-sample items A1 in rounds ran 10 968 instead of 23 729, each
        // item's fixed costs beside a one-ray path (profiles/r06/ab_A2_round_items.txt).
        // Item sizes are scheduling only: the combine folds every sample in order.
        unsigned long long rays = 0, paths = 0;
        if (round && P->counters) {
            rays = P->counters[C_RAYS];
            paths = P->counters[C_PATHS];
            P->rpp_hint[0] = rays;
            P->rpp_hint[1] = paths;
        } else if (!round) {
            rays = P->rpp_hint[0];
            paths = P->rpp_hint[1];
        }
        if (paths && rays >= 2ull * paths) {
            csz = 1u;
        } else {
            csz = min(16u, bs);
            while (csz > 1u && (uint64_t)n_seg * ((bs + csz - 1u) / csz) < 8ull * P->lanes) csz >>= 1;
        }
    }
    const uint32_t cpp = whole ? 1u : (bs + csz - 1u) / csz;
    P->per_sample = whole ? 0u : 1u;
    P->chunk = whole ? 0u : csz;
    P->round = round;
    P->cpp = cpp;
    P->u_cpp = udiv_make(cpp);
    P->n_items = n_seg * cpp;
    P->fine_base = 0xFFFFFFFFu;  // no fine region
    P->fine_px = P->capacity;
    // (items of a few samples claim more at a time, as fine chunks do: the one queue counter
    // serialises the claims, and a tail round runs millions of 1-sample items)
    P->claim = max(1u, min(whole || csz > 4u ? 32u : (uint32_t)GS_CLAIM_FINE,
                           P->n_items / max(1u, P->waves) / (uint32_t)GS_CLAIM_DIV));
    P->claim_fine = P->claim;
    P->round_base = round * bs;
    P->seg_base = base;
    P->seg_n = n_seg;
    P->active = P->active_buf[round & 1u];
    P->next_active = P->active_buf[(round & 1u) ^ 1u];
    *P->queue = 0u;
}

// After each (round, segment) launch: per active pixel, its batch folded into the running
// sums in sample order (camera.rs:142-146), then the stop test (:149-164) exactly as the
// per-lane loop takes it; a stopped pixel's colour (:167) is written, the rest go on.
__global__ void gs_round_combine_kernel(const KParams* __restrict__ P, uint32_t round) {
    if (!P->per_sample) return;  // a whole-batch round: the lanes took the stop test
    const uint32_t n = P->seg_n, bs = P->ss.batch_size, lane = threadIdx.x & 63u;
    const uint32_t span = (n + 63u) & ~63u;
    const double confidence_sq = P->ss.confidence * P->ss.confidence;
    const double tolerance_sq = P->ss.tolerance * P->ss.tolerance;
    // sample_count after this round's batch: 0.0 + bs + bs + ... (exact: integers < 2^53)
    const double scount = (double)((uint64_t)(round + 1u) * bs);
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < span; a += gridDim.x * blockDim.x) {
        bool go_on = false, stopped = false;
        uint32_t item = 0;
        if (a < n) {
            item = P->active[P->seg_base + a];
            double* ps = P->pstate + (size_t)item * 5;
            double r = 0.0, g = 0.0, b = 0.0, lsum = 0.0, lsq = 0.0;
            if (round) {
                r = ps[0];
                g = ps[1];
                b = ps[2];
                lsum = ps[3];
                lsq = ps[4];
            }
            const double* smp = P->partial + (size_t)a * (GS_ROUND_PIXEL_MAJOR ? bs : 1u) * 3;
            for (uint32_t j = 0; j < bs; j++, smp += (GS_ROUND_PIXEL_MAJOR ? 1u : (size_t)n) * 3) {
                const double cr = smp[0], cg = smp[1], cb = smp[2];
                r += cr;
                g += cg;
                b += cb;
                const double lum = 0.299 * cr + 0.587 * cg + 0.144 * cb;
                lsum += lum;
                lsq += lum * lum;
            }
            const double mean = lsum / scount;
            const double variance_sq = 1.0 / (scount - 1.0) * (lsq - lsum * lsum / scount);
            const double convergence_sq = confidence_sq * variance_sq / scount;
            bool stop = convergence_sq < (mean * mean * tolerance_sq);
            if (!stop) stop = (uint32_t)sat_u64(scount, 4294967295.0, 4294967295ull) > P->ss.max_samples;
            if (stop) {
                const double cr = r / scount, cg = g / scount, cb = b / scount;
                uint32_t pi = 0, pj = 0;
                if (P->direct) (void)packed_pixel(P, item, pi, pj);  // (an active pixel is real)
                const size_t oi = P->direct ? (size_t)pj * (uint32_t)P->cam.image_width + pi : (size_t)item;
                if (P->out) {
                    float* o = P->out + oi * 3;
                    o[0] = (float)cr;
                    o[1] = (float)cg;
                    o[2] = (float)cb;
                }
                if (P->out8) {
                    uint8_t* o8 = P->out8 + oi * 3;
                    o8[0] = color_byte(cr);
                    o8[1] = color_byte(cg);
                    o8[2] = color_byte(cb);
                }
                stopped = true;
            } else {
                ps[0] = r;
                ps[1] = g;
                ps[2] = b;
                ps[3] = lsum;
                ps[4] = lsq;
                go_on = true;
            }
        }
        const uint64_t mg = __builtin_amdgcn_ballot_w64(go_on), ms = __builtin_amdgcn_ballot_w64(stopped);
        if (mg != 0) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(mg);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(&P->round_counts[round + 1u], (uint32_t)__popcll(mg));
            base = __shfl(base, (int)leader);
            if (go_on) P->next_active[base + (uint32_t)__popcll(mg & ((1ull << lane) - 1ull))] = item;
        }
        if (ms != 0 && P->counters && lane == (uint32_t)__builtin_ctzll(ms))
            atomicAdd(&P->counters[C_PIX], (unsigned long long)__popcll(ms));
    }
}

// =============================================================== host side
static thread_local std::string tl_err;
// Process-wide tuning (the gs_set_* / gs_debug_set_* setters).  Atomics: a setter may run
// while another thread launches; each launch reads every value once, so
// one launch never mixes two settings of the same knob.
static std::atomic<int32_t> g_shade_batch{0};   // 0: the scene's own (52, or GS_KIND_SHADE_BATCH with BVHs under instances);  // swept on MI355X C4 (chunked, uniform loop): 48 -> 3502, 52 -> 3535-3568, 56 -> 3506-3536 Msamples/s
static std::atomic<int32_t> g_blocks_per_cu{0};  // 0 = occupancy query
static std::atomic<int32_t> g_node_steps{0};  // 0: the scene's own (gs_device_scene.node_steps)
// leaf batch: 0 = the scene's choice (12: swept on MI355X C4 with leaf runs: 8 -> 4586, 10 ->
// 4632, 12 -> 4648-4651, 14 -> 4624, 16 -> 4592; GS_KIND_LEAF_BATCH for kind-batched kernels)
static std::atomic<int32_t> g_leaf_batch{0};
static std::atomic<int32_t> g_cam_batch{0};  // 0: the scene's own (gs_set_camera_batch)
static std::atomic<int32_t> g_tail_pct{0};  // guided tail (gs_debug_set_guided_tail): 0 = default
#ifndef GS_KIND_SHADE_BATCH
#define GS_KIND_SHADE_BATCH 44
#endif
#ifndef GS_KIND_LEAF_BATCH
#define GS_KIND_LEAF_BATCH 24
#endif
#ifndef GS_KIND_NODE_STEPS
#define GS_KIND_NODE_STEPS 8
#endif
// Bytes of threaded records mirrored in LDS per block (the most-tested ones): what is
// left of the block's share of the CU's 160 KiB (4 waves/SIMD = 1024 lanes per CU) after
// the lane state.  -1 = that budget; >= 0 explicit (A/B).
#ifndef GS_LDS_MIRROR
#define GS_LDS_MIRROR -1
#endif
static const int64_t g_lds_mirror = GS_LDS_MIRROR;  // (compile-time A/B only)
static int64_t lds_mirror_budget() {
    const int64_t share = (int64_t)160 * 1024 * GS_BLOCK / (GS_MIN_WAVES * 4 * 64);  // the block's share of the CU
    // (sized for fixed-spp launches; an adaptive launch's larger lane state shrinks the
    // mirror's prefixes to fit at launch)
    const int64_t left = share - (int64_t)GS_BLOCK * (L_ND_CHUNKED * 8 + L_NI * 4) - 1024;  // 1 KiB: static LDS + slack
    return left > 0 ? left : 0;
}
// -1 auto, 0 never split a pixel's samples.  Swept on MI355X with batched queue claims,
// C4 rank 0 / rank 3 of N (tools/rank_sim.py; ms): N=1: 4 -> 658.4, 8 -> 658.7,
// 16 -> 648.3, 32 -> 647.3; N=8: 4 -> 89.6, 8 -> 89.6, 16 -> 89.7, 32 -> 95.8 (max of the
// two ranks).  16 is within noise of the best at both ends.
static std::atomic<int32_t> g_sample_chunk{-1};
static std::atomic<int32_t> g_placement{1};  // 1: placement pilot at a scene's first launch; 0: the static estimate only
static std::atomic<uint64_t> g_partial_budget{4ull << 30};  // auto chunks: at most 4 GiB of chunk sums (per launch slot)
// Adaptive settings (more than one batch): 1 = batch rounds (gs_round_*_kernel), 0 = the
// per-lane loop (one work item per pixel running every batch).  Bit-identical results.
static std::atomic<int32_t> g_adaptive_rounds{1};  // 1 auto (GS_ROUND_MIN_CAP), 2 always rounds, 0 never
// Work items of a round: 0 split (default; measured on MI355X, A2 cornell_box 1024^2: split
// 7520, whole-batch items while the active pixels fill the lanes twice 5910 Msamples/s;
// A1 hdri 19738 vs 18124), 1 whole-batch items, -1 whole while the active pixels fill the
// lanes twice.
static std::atomic<int32_t> g_round_whole{0};
// Auto mode: batch rounds when a pixel can take at least this many samples ((max_samples /
// batch + 1) x batch): the per-lane loop's tail is up to that many samples in one lane.
// MI355X: A2 cornell_box (cap 1024) rounds 7520 vs per-lane 5394 Msamples/s; A1 hdri (cap
// 256) rounds 19738 vs per-lane 24582 -- its pixels stop after one or two batches, and the
// rounds' per-sample colours and launches cost more than its short tail.
#ifndef GS_ROUND_MIN_CAP
#define GS_ROUND_MIN_CAP 512
#endif
static const uint64_t kMaxRounds = 1u << 16;  // more batches than this: the per-lane loop

extern "C" void gs_set_last_error(const char* msg) { tl_err = msg ? msg : ""; }
static gs_status fail(gs_status code, const std::string& msg) {
    tl_err = msg;
    return code;
}
#define HIPCHK(x)                                                                               \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) return fail(GS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// One in-flight launch's device state: its parameter block, its work-queue counter and
// its chunk sums.  A scene keeps a small ring of them, so launches of one scene on
// different streams (or host threads) never share state; a slot is reused only after
// the stream of the new launch has waited for the slot's previous launch (its event).
struct LaunchSlot {
    KParams* params = nullptr;  // device
    uint32_t* queue = nullptr;  // device
    double* partial = nullptr;  // chunk partial sums, grown on demand
    size_t partial_bytes = 0;
    hipEvent_t done = nullptr;  // recorded after the slot's last launch
    hipStream_t stream = nullptr;  // the stream of the slot's last launch
    bool used = false;
    // batch rounds (adaptive settings): round counts, the two active lists, the running sums
    void* rbuf = nullptr;
    size_t rbuf_bytes = 0;
    // GS_FEAT_NESTED: each lane's save slots (KParams::nest_save), 8 slot-major arrays of 8 B per lane of the grid
    double* nest_save = nullptr;
    size_t nest_save_bytes = 0;
};
static const int kLaunchSlots = 4;

// The threaded top-level tree before placement: pre-order records (DNode: a node's f64
// box, hit link = the next record, miss link; a leaf's sphere inline, next link, ABI ref),
// with each record's depth and static visit estimate.
struct ThreadedTree {
    std::vector<DNode> rec;
    std::vector<uint8_t> leaf;
    std::vector<uint32_t> depth;
    std::vector<double> score;
};
struct gs_device_scene {
    int device = 0;
    void* mem = nullptr;  // one allocation for every array
    size_t bytes = 0;
    DevScene dev{};
    uint32_t n_nodes = 0;
    uint32_t bvh_depth = 1;  // top-level BVH depth (informational: the walk keeps no stack)
    bool cert_boxes = false;  // every top-level node coordinate |x| <= 1e15 (box_cert applies)
    int feat = 0;             // GS_FEAT_* of the kernel instantiation to launch
    // The threaded top-level tree (THR_*): node records, their f64 boxes, leaf records.
    const TNode* tnodes = nullptr;
    const TBox* tboxes = nullptr;
    const TLeaf* tleaves = nullptr;
    const TQuad* tquads = nullptr;  // every quad's traversal record, gs_quad order
    uint32_t thr_root = THR_END;
    uint32_t lds_nodes = 0, lds_leaves = 0, lds_quads = 0;  // mirrored prefixes (per block)
    // BVHs under instance chains, threaded into the node / leaf arrays with the top-level
    // tree: each tree's root record (tree index -> record of ThreadedTree), and the device
    // array of their links (DevScene::nroots), rewritten with the records at re-placement
    std::vector<uint32_t> nroot_rec;
    uint32_t* nroots = nullptr;
    uint32_t n_cubes = 0, lds_cubes = 0;  // Quad::cube records (cube_test), and the mirrored prefix
    int32_t node_steps = GS_NODE_STEPS;      // node steps per node pass (from the tree's shape)
    int32_t leaf_batch = 12;                 // lanes at a leaf before a leaf pass (scene's choice)
    int32_t shade_batch = 52;                // finished lanes a wave shades together (scene's choice)
    int32_t cam_batch = 1;                   // lanes waiting for camera rays before a wave runs get_ray
    // A sample's cost on this device, lane-microseconds (kernel time x lanes / samples), from
    // the frame context's last frame (gs_device_scene_note_frame); 0 = not measured yet.  Once
    // a frame measured long samples, the guided tail's small-frame rule stays off for the
    // scene (long_samples: sticky, so a scene near the threshold does not alternate layouts
    // from frame to frame).
    std::atomic<double> lane_us_per_sample{0.0};
    std::atomic<bool> long_samples{false};
    uint32_t node_records = 0, leaf_records = 0;
    double nodes_per_leaf = 0.0, other_leaf_frac = 0.0;
    // Launch state, mutated by launches of a const scene: guarded by `mu`.
    std::mutex mu;
    // launch geometry, computed at the first launch (host API queries cost ~0.5 ms each)
    // Launch shape per lane-state layout ([1]: fixed-spp / chunked launches, [0]: adaptive):
    // the mirror prefixes that fit next to that lane state, the dynamic LDS, the kernel
    // instantiation (feat minus GS_FEAT_LDSTREE when the mirror is a strict prefix), blocks/CU.
    struct LaunchCfg {
        bool ready = false;
        uint32_t lds_nodes = 0, lds_leaves = 0, lds_quads = 0, lds_cubes = 0, nest_lds = 0;
        size_t lds = 0;
        int feat = 0, per_cu = 0;
    } lcfg[2];
    int cus = 0;
    LaunchSlot slots[kLaunchSlots];
    uint32_t next_slot = 0;
    // Placement of the threaded records (place_records): the static estimate until the
    // first launch, whose pilot (run_pilot) measures the visits and re-places them.
    ThreadedTree tree;
    std::vector<uint32_t> pos;  // tree record -> position (current placement)
    uint32_t n_quads = 0;
    std::vector<uint32_t> single_quads;  // the quads outside cube lists (place_records)
    int64_t mirror_budget = 0;
    std::atomic<int> placement{0};  // 0 static, pilot pending; 1 static (final); 2 measured
    double pilot_ms = 0.0;
    std::mutex place_mu;  // held while a pilot runs and the records are re-placed
};

namespace {

struct Layout {
    std::vector<uint8_t> blob;
    size_t add(const void* p, size_t n) {
        size_t off = (blob.size() + 255) & ~(size_t)255;
        blob.resize(off + n + 1, 0);  // +1 keeps empty arrays at distinct, valid addresses
        if (n && p) std::memcpy(blob.data() + off, p, n);
        return off;
    }
};

// The device arrays of one placement: node records, their f64 boxes, leaf records, with
// the mirrored prefixes first, and the root's link.
struct Placed {
    std::vector<TNode> tnodes;
    std::vector<TBox> tboxes;
    std::vector<TLeaf> tleaves;
    std::vector<uint32_t> pos;  // tree record -> its position in tnodes / tleaves
    std::vector<uint32_t> nroots;  // the links of the nested trees' roots (DevScene::nroots)
    uint32_t lds_nodes = 0, lds_leaves = 0, lds_quads = 0, lds_cubes = 0, root = THR_END;
};
// Order the records by how likely a ray tests them and fill the block's LDS byte budget in
// that order (32-B node records, 48-B leaf records; quads take the rest).  `visits` (one
// count per record, nullable): measured by a pilot launch (GS_FEAT_VISITS), ranked by
// visits per byte, which maximises the visits the mirror serves; the static estimate
// orders the unvisited and serves when there is no pilot.  Records outside the mirror
// stay in pre-order.
// The aligned form of a quad (cube_record) when its normal is
// exactly +-e_a, w is zero off axis a, and u, v are each non-zero on one other axis.
static bool aligned_tquad(const gs_quad& q, TQuad& out) {
    int ax = -1;
    for (int k = 0; k < 3; k++) {
        if (q.normal[k] == 0.0) continue;
        if (std::fabs(q.normal[k]) != 1.0 || ax >= 0) return false;
        ax = k;
    }
    if (ax < 0) return false;
    auto one_axis = [&](const double* v) {
        int at = -1;
        for (int k = 0; k < 3; k++) {
            if (!std::isfinite(v[k])) return -2;
            if (v[k] != 0.0) {
                if (at >= 0) return -2;
                at = k;
            }
        }
        return at;
    };
    const int iu = one_axis(q.u), iv = one_axis(q.v);
    if (iu < 0 || iv < 0 || iu == ax || iv == ax || iu == iv) return false;
    for (int k = 0; k < 3; k++)
        if (k != ax && q.w[k] != 0.0) return false;
    if (!std::isfinite(q.w[ax]) || !std::isfinite(q.d) || !std::isfinite(q.q[iu]) || !std::isfinite(q.q[iv])) return false;
    const int o = iu == (ax + 1) % 3 ? 0 : 1;  // (then iv == (ax + 2) % 3 for o == 0)
    const double sgn = o == 0 ? 1.0 : -1.0;
    TQuad r{};
    const uint64_t tag = ((uint64_t)(GS_AQ_TAG | (uint32_t)(2 * ax + o))) << 32;
    std::memcpy(&r.nx, &tag, 8);
    r.ny = q.normal[ax] * q.d;  // D' (exact: a sign)
    r.nz = q.q[iu];
    r.d = q.q[iv];
    r.qx = q.u[iu];
    r.qy = q.v[iv];
    r.qz = sgn * q.w[ax];  // W'
    out = r;
    return true;
}

static std::atomic<int32_t> g_cube_lists{1};  // gs_debug_set_cube_lists
#ifndef GS_PLAIN_KERNELS
#define GS_PLAIN_KERNELS 1  // (A/B: 0 keeps C4 on the generic staged shading)
#endif
static const bool g_plain_kernels = GS_PLAIN_KERNELS;
// A Quad::cube list's device record (cube_test): six consecutive quads whose aligned forms
// carry cube_code(k) in order and equal, field by field, what cube_src derives from the 12
// numbers taken from them.  Returns false (the list keeps the loop) otherwise.
static bool cube_record(const gs_flat_scene& s, const gs_list& l, uint32_t& q0, double* out) {
    if (l.count != 6 || (uint64_t)l.first + 6 > s.n_list_refs) return false;
    q0 = s.list_refs[l.first] & GS_REF_MASK;
    if (q0 >= GS_CUBE_FLAG) return false;
    double f[6][6];  // face k: D', Q_iu, Q_iv, U_iu, V_iv, W'
    for (uint32_t k = 0; k < 6; k++) {
        const uint32_t ref = s.list_refs[l.first + k];
        if ((ref >> GS_REF_SHIFT) != GS_REF_QUAD || (ref & GS_REF_MASK) != q0 + k || q0 + k >= s.n_quads) return false;
        TQuad a;
        if (!aligned_tquad(s.quads[q0 + k], a)) return false;
        uint64_t tag;
        std::memcpy(&tag, &a.nx, 8);
        if ((uint32_t)(tag >> 32) != (GS_AQ_TAG | (uint32_t)cube_code((int)k))) return false;
        const double v[6] = {a.ny, a.nz, a.d, a.qx, a.qy, a.qz};
        for (int j = 0; j < 6; j++) f[k][j] = v[j];
    }
    // x0 y0 z0 x1 y1 z1 dx dy dz w_xy w_zy w_xz, read off faces 3, 5, 2, 1, 4, 0 (cube_src)
    const double c[GS_CUBE_DOUBLES] = {f[3][0], f[5][0], f[2][0], f[1][0], f[4][0], f[0][0],
                                       f[0][3], f[0][4], f[3][3], f[0][5], f[3][5], f[5][5]};
    for (int k = 0; k < 6; k++)
        for (int j = 0; j < 6; j++) {
            const int v = cube_src(k, j);
            if (!(f[k][j] == (v < 0 ? -c[-v] : c[v]))) return false;
        }
    for (int j = 0; j < GS_CUBE_DOUBLES; j++) out[j] = c[j];
    return true;
}

// Raw links of ThreadedTree records: a record index, or the end of the top-level walk, or
// the end of a nested tree's walk (THR_END / THR_RET once placed).
#define RAW_END 0xFFFFFFFFu
#define RAW_RET 0xFFFFFFFEu
static Placed place_records(const ThreadedTree& t, const std::vector<uint64_t>* visits,
                            const std::vector<uint32_t>& single_quads, int64_t budget,
                            const std::vector<uint32_t>& nroot_rec, uint32_t n_cubes) {
    const uint32_t n = (uint32_t)t.rec.size();
    Placed out;
    std::vector<uint32_t> order(n), pos(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    auto rec_bytes = [&](uint32_t i) { return t.leaf[i] ? (int64_t)sizeof(TLeaf) : (int64_t)sizeof(TNode); };
    auto static_first = [&](uint32_t a, uint32_t b) {
        return t.score[a] > t.score[b] || (t.score[a] == t.score[b] && t.depth[a] < t.depth[b]);
    };
    if (visits) {
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
            // compare visits_a / bytes_a with visits_b / bytes_b exactly (integers)
            const unsigned __int128 va = (unsigned __int128)(*visits)[a] * (uint64_t)rec_bytes(b);
            const unsigned __int128 vb = (unsigned __int128)(*visits)[b] * (uint64_t)rec_bytes(a);
            if (va != vb) return va > vb;
            return static_first(a, b);
        });
    } else {
        std::stable_sort(order.begin(), order.end(), static_first);
    }
    std::vector<uint8_t> top(n, 0);
    int64_t used = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t r = order[i];
        const int64_t sz = rec_bytes(r);
        if (used + sz > budget) {
            if (used + (int64_t)sizeof(TNode) > budget) break;
            continue;
        }
        used += sz;
        top[r] = 1;
        (t.leaf[r] ? out.lds_leaves : out.lds_nodes)++;
    }
    // (the nested trees' records are ranked with the top level's: one node / leaf array)
    // a prefix of the quads up to the last quad tested by the quad test that fits (cube-list
    // quads are read from the cube records)
    const int64_t fit = std::max<int64_t>(0, budget - used) / (int64_t)sizeof(TQuad);
    out.lds_quads = 0;
    for (uint32_t q : single_quads)
        if ((int64_t)q < fit) out.lds_quads = q + 1;
    used += (int64_t)out.lds_quads * (int64_t)sizeof(TQuad);
    // then the Quad::cube records (cube order)
    out.lds_cubes = (uint32_t)std::min<int64_t>(n_cubes, std::max<int64_t>(0, budget - used) / (GS_CUBE_DOUBLES * 8));
    // The mirrored records take their positions in rank order, so a launch that must
    // shrink the prefixes (a larger lane state, gs_render_tiles_timed_async) drops the
    // least-tested ones; the rest keep pre-order.
    uint32_t nt = 0, nl = 0, nt_rest = out.lds_nodes, nl_rest = out.lds_leaves;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t i = order[k];
        if (top[i]) pos[i] = t.leaf[i] ? nl++ : nt++;
    }
    for (uint32_t i = 0; i < n; i++)
        if (!top[i]) pos[i] = t.leaf[i] ? nl_rest++ : nt_rest++;
    out.tnodes.resize(nt_rest);
    out.tboxes.resize(nt_rest);
    out.tleaves.resize(nl_rest);
    auto tag = [&](uint32_t l) {
        if (l == RAW_RET) return THR_RET;
        return l >= n ? THR_END : (t.leaf[l] ? (THR_LEAF | pos[l]) : node_link(pos[l]));
    };
    for (uint32_t i = 0; i < n; i++) {
        const DNode& r = t.rec[i];
        if (t.leaf[i]) {
            out.tleaves[pos[i]] = TLeaf{r.mnx, r.mny, r.mnz, r.mxx * r.mxx, tag(r.left), r.right, 0u, 0u};
        } else {
            // f32 box coordinates rounded to nearest (the certified test's error model)
            out.tnodes[pos[i]] = TNode{(float)r.mnx, (float)r.mny, (float)r.mxx, (float)r.mxy, (float)r.mnz,
                                       (float)r.mxz, tag(r.left), tag(r.right)};
            out.tboxes[pos[i]] = TBox{r.mnx, r.mny, r.mnz, r.mxx, r.mxy, r.mxz};
        }
    }
    out.root = n == 0 ? THR_END : tag(0);
    for (uint32_t r : nroot_rec) out.nroots.push_back(tag(r));
    out.pos = std::move(pos);
    return out;
}

// Host-side validation of everything the kernel indexes, so a malformed scene is an
// error code, never a GPU fault.
// inst_reached (out): per instance, whether a leaf reachable from the root walks it (the scene
// upload threads the BVHs under reached instances only).
gs_status validate(const gs_flat_scene& s, uint32_t* depth_out, bool* nested_out, std::vector<uint8_t>* inst_reached,
                   bool* general_out, std::vector<uint8_t>* media_reached) {
    media_reached->assign(s.n_media, 0);
    bool general = false;  // a composition only GS_FEAT_GENERAL kernels walk (round 6)
    auto bad = [](const std::string& m) { return fail(GS_ERR_ARG, "invalid flat scene: " + m); };
    auto unsup = [](const std::string& m) { return fail(GS_ERR_UNSUPPORTED, m); };
    if (!s.nodes && s.n_nodes) return bad("nodes");
    if (!s.media && s.n_media) return bad("media");
    // the kernel forms node / sphere byte offsets as u32 (ref << 6, ref << 5)
    if (s.n_nodes >= (1u << 26) || s.n_spheres >= (1u << 27)) return unsup("more than 2^26 BVH nodes or 2^27 spheres");
    if (s.n_materials == 0 || !s.materials) return bad("no materials");
    if (!s.instances && s.n_instances) return bad("instances");
    inst_reached->assign(s.n_instances, 0);
    auto prim_ok = [&](uint32_t r) {
        uint32_t k = r >> GS_REF_SHIFT, i = r & GS_REF_MASK;
        switch (k) {
            case GS_REF_SPHERE: return i < s.n_spheres;
            case GS_REF_MSPHERE: return i < s.n_mspheres;
            case GS_REF_QUAD: return i < s.n_quads;
            case GS_REF_TRIANGLE: return i < s.n_triangles;
            default: return false;
        }
    };
    // Walks a Translate/RotateY chain: 0 ok, 1 bad, 2 unsupported (deeper than GS_MAX_CHAIN).
    // mark: 1 a leaf's chain, 2 a medium boundary's (kept: a chain reached both ways is 2)
    auto chain_ok = [&](uint32_t& cur, uint8_t mark = 1) -> int {
        int chain = 0;
        while ((cur >> GS_REF_SHIFT) == GS_REF_INSTANCE) {
            uint32_t i = cur & GS_REF_MASK;
            if (i >= s.n_instances) return 1;
            if (++chain > GS_MAX_CHAIN) return 2;
            if (chain > 4) general = true;  // (the other kernels' hit record keeps 4)
            (*inst_reached)[i] = std::max((*inst_reached)[i], mark);
            const gs_instance& in = s.instances[i];
            if (in.kind != GS_INST_TRANSLATE && in.kind != GS_INST_ROTATE_Y) return 1;
            cur = in.child;
        }
        return 0;
    };
    // A list of primitives or one primitive (what walk_chain may end in).
    auto shape_ok = [&](uint32_t cur) -> int {
        const uint32_t k = cur >> GS_REF_SHIFT;
        if (k == GS_REF_LIST) {
            uint32_t i = cur & GS_REF_MASK;
            if (i >= s.n_lists) return 1;
            const gs_list& l = s.lists[i];
            if ((uint64_t)l.first + l.count > s.n_list_refs) return 1;
            for (uint32_t q = 0; q < l.count; q++)
                if (!prim_ok(s.list_refs[l.first + q])) return 2;
            return 0;
        }
        if (k == GS_REF_NODE || k == GS_REF_MEDIUM || k == GS_REF_INSTANCE) return 2;
        return prim_ok(cur) ? 0 : 1;
    };
    // A BVH under an instance chain: nodes in range, leaves lists or primitives, depth at
    // most GS_NESTED_STACK (the device walk is threaded and needs no stack; the bound keeps
    // the host's threading finite).  Subtrees may be shared between chains (instancing);
    // the depth bound ends cycles and a visit budget ends blow-ups.
    // A BVH as a medium boundary (GS_FEAT_GENERAL, tree_test): nodes in range, leaves lists or
    // primitives, depth bounded (threaded with the BVHs under instances).
    uint64_t boundary_budget = 64ull << 20;
    auto boundary_tree_ok = [&](uint32_t root) -> int {
        std::vector<std::pair<uint32_t, uint32_t>> st{{root, 1u}};
        while (!st.empty()) {
            auto [r, d] = st.back();
            st.pop_back();
            if (boundary_budget-- == 0) return 1;
            if ((r >> GS_REF_SHIFT) == GS_REF_NODE) {
                const uint32_t i = r & GS_REF_MASK;
                if (i >= s.n_nodes) return 1;
                if (d > GS_NESTED_STACK) return 2;
                if (s.nodes[i].left == GS_REF_NONE) return 1;
                st.push_back({s.nodes[i].left, d + 1});
                if (s.nodes[i].right != GS_REF_NONE) st.push_back({s.nodes[i].right, d + 1});
            } else {
                const int e = shape_ok(r);
                if (e) return e;
            }
        }
        return 0;
    };
    // A ConstantMedium: its boundary a primitive or list behind an optional chain; round 6
    // (GS_FEAT_GENERAL): also a BVH, or one level of another medium.
    std::function<int(uint32_t, int)> medium_ok_l = [&](uint32_t cur, int level) -> int {
        uint32_t i = cur & GS_REF_MASK;
        if (i >= s.n_media || !s.media) return 1;
        if (s.media[i].material >= s.n_materials) return 1;
        uint32_t b = s.media[i].boundary;
        const int e = chain_ok(b, 2);
        (*media_reached)[i] = 1;
        if (e) return e;
        if ((b >> GS_REF_SHIFT) == GS_REF_NODE) {
            general = true;
            return boundary_tree_ok(b);
        }
        if ((b >> GS_REF_SHIFT) == GS_REF_MEDIUM) {
            if (level > 0) return 2;  // media two deep inside media
            general = true;
            return medium_ok_l(b, level + 1);
        }
        return shape_ok(b);
    };
    auto medium_ok = [&](uint32_t cur) -> int { return medium_ok_l(cur, 0); };
    bool nested = false;
    uint64_t nested_budget = 64ull << 20;
    auto nested_ok = [&](uint32_t root) -> int {
        std::vector<std::pair<uint32_t, uint32_t>> st{{root, 1u}};
        while (!st.empty()) {
            auto [r, d] = st.back();
            st.pop_back();
            if (nested_budget-- == 0) return 1;
            if ((r >> GS_REF_SHIFT) == GS_REF_NODE) {
                const uint32_t i = r & GS_REF_MASK;
                if (i >= s.n_nodes) return 1;
                if (d > GS_NESTED_STACK) return 2;
                if (s.nodes[i].left == GS_REF_NONE) return 1;
                st.push_back({s.nodes[i].left, d + 1});
                if (s.nodes[i].right != GS_REF_NONE) st.push_back({s.nodes[i].right, d + 1});
            } else {
                // (since round 5 the tree is walked by the main passes, whose leaf test takes
                // media like the top level's: the hit's instance is the tree's chain; round 6: a
                // chain inside the tree, ending in a primitive, list or medium -- not another BVH)
                uint32_t c = r;
                int e = chain_ok(c);
                if (!e) {
                    if (c != r) general = true;  // a chain inside the tree: two-chain hit records
                    if ((c >> GS_REF_SHIFT) == GS_REF_NODE) e = 2;
                    else e = (c >> GS_REF_SHIFT) == GS_REF_MEDIUM ? medium_ok(c) : shape_ok(c);
                }
                if (e) return e;
            }
        }
        nested = true;
        return 0;
    };
    auto leaf_ok = [&](uint32_t r) -> int {  // 0 ok, 1 bad, 2 unsupported
        uint32_t cur = r;
        int e = chain_ok(cur);
        if (e) return e;
        if ((cur >> GS_REF_SHIFT) == GS_REF_NODE && cur != r) return nested_ok(cur);
        if ((cur >> GS_REF_SHIFT) == GS_REF_MEDIUM) return medium_ok(cur);
        if ((cur >> GS_REF_SHIFT) == GS_REF_NODE) return cur != r ? 2 : 1;
        return shape_ok(cur);
    };
    // Walk the tree from the root: indices in range, no node reached twice, depth bound.
    std::vector<uint8_t> seen(s.n_nodes, 0);
    std::vector<std::pair<uint32_t, uint32_t>> stk;
    stk.push_back({s.root, 0});
    uint32_t maxd = 0;
    while (!stk.empty()) {
        auto [r, d] = stk.back();
        stk.pop_back();
        if ((r >> GS_REF_SHIFT) == GS_REF_NODE) {
            uint32_t i = r & GS_REF_MASK;
            if (i >= s.n_nodes) return bad("node index");
            if (seen[i]) return bad("node reached twice (not a tree)");
            seen[i] = 1;
            if (d + 1 > maxd) maxd = d + 1;
            if (s.nodes[i].left == GS_REF_NONE) return bad("node without left child");
            stk.push_back({s.nodes[i].left, d + 1});
            if (s.nodes[i].right != GS_REF_NONE) stk.push_back({s.nodes[i].right, d + 1});
        } else {
            int e = leaf_ok(r);
            if (e == 1) return bad("leaf reference");
            if (e == 2) return unsup("instance chain deeper than " + std::to_string(GS_MAX_CHAIN) +
                                     ", a BVH under an instance deeper than " + std::to_string(GS_NESTED_STACK) +
                                     " or holding another BVH under an instance, a BVH inside a medium boundary, "
                                     "nested media, or a list member that is not a primitive");
        }
    }
    *depth_out = maxd;
    *nested_out = nested;
    *general_out = general;
    auto mat_ok = [&](uint32_t m) { return m < s.n_materials; };
    for (uint32_t i = 0; i < s.n_spheres; i++) if (!mat_ok(s.spheres[i].material)) return bad("sphere material");
    for (uint32_t i = 0; i < s.n_mspheres; i++) if (!mat_ok(s.mspheres[i].material)) return bad("msphere material");
    for (uint32_t i = 0; i < s.n_quads; i++) if (!mat_ok(s.quads[i].material)) return bad("quad material");
    for (uint32_t i = 0; i < s.n_triangles; i++) if (!mat_ok(s.triangles[i].material)) return bad("triangle material");
    for (uint32_t i = 0; i < s.n_materials; i++) {
        const gs_material& m = s.materials[i];
        if (m.kind == GS_MAT_LAMBERTIAN || m.kind == GS_MAT_DIFFUSE_LIGHT || m.kind == GS_MAT_ISOTROPIC) {
            if (m.texture >= s.n_textures) return bad("material texture");
        } else if (m.kind != GS_MAT_METAL && m.kind != GS_MAT_DIELECTRIC) {
            return bad("material kind");
        }
    }
    for (uint32_t i = 0; i < s.n_textures; i++) {
        const gs_texture& t = s.textures[i];
        if (t.kind == GS_TEX_CHECKERED) {
            if (t.even >= s.n_textures || t.odd >= s.n_textures) return bad("checkered child");
        } else if (t.kind == GS_TEX_IMAGE) {
            if (t.image >= s.n_images) return bad("image index");
            const gs_image& im = s.images[t.image];
            if (!im.width || !im.height) return bad("empty image");
            if (im.offset + (uint64_t)im.width * im.height * 3 > s.n_texels8) return bad("image texels out of range");
        } else if (t.kind == GS_TEX_NOISE) {
            if (s.n_noise_perm != 256 || !s.noise_perm) return bad("noise texture without its 256-byte permutation");
        } else if (t.kind != GS_TEX_SOLID) {
            return bad("texture kind");
        }
    }
    if (s.background.kind == GS_BG_HDRI) {
        if (!s.background.width || !s.background.height) return bad("empty HDRI");
        if ((uint64_t)s.background.width * s.background.height * 3 > s.n_hdri_floats || !s.hdri_rgb)
            return bad("HDRI texels");
    } else if (s.background.kind != GS_BG_SOLID) {
        return bad("background kind");
    }
    return GS_OK;
}

// f32 RGB -> RGBE8 (shared exponent), accepted only if m * 2^(e-136) reproduces all
// three floats exactly (true for texels that came from an RGBE file, as airport.hdr's).
bool encode_rgbe(const float* c, uint32_t* out) {
    const float r = c[0], g = c[1], b = c[2];
    if (!(r >= 0.0f && g >= 0.0f && b >= 0.0f)) return false;
    if (std::signbit(r) || std::signbit(g) || std::signbit(b)) return false;
    const float mx = std::fmax(r, std::fmax(g, b));
    if (mx == 0.0f) {
        *out = 0;
        return true;
    }
    int ex = 0;
    std::frexp((double)mx, &ex);
    for (int e = ex + 128; e >= 1 && e >= ex + 120; e--) {  // try the canonical exponent first
        if (e > 255) continue;
        const double scale = std::ldexp(1.0, e - 136);
        uint32_t m[3];
        bool ok = true;
        for (int k = 0; k < 3 && ok; k++) {
            const double q = (double)c[k] / scale;
            ok = q >= 0.0 && q <= 255.0 && q == std::floor(q) && (float)(q * scale) == c[k];
            m[k] = ok ? (uint32_t)q : 0;
        }
        if (ok) {
            *out = m[0] | (m[1] << 8) | (m[2] << 16) | ((uint32_t)e << 24);
            return true;
        }
    }
    return false;
}

// Does the texture tree under `t` contain an image (=> sphere uv must be computed)?
bool tex_needs_uv(const gs_flat_scene& s, uint32_t t, int depth = 0) {
    if (t >= s.n_textures || depth > 16) return false;
    const gs_texture& x = s.textures[t];
    if (x.kind == GS_TEX_IMAGE) return true;
    if (x.kind == GS_TEX_CHECKERED) return tex_needs_uv(s, x.even, depth + 1) || tex_needs_uv(s, x.odd, depth + 1);
    return false;
}

}  // namespace

extern "C" {

const char* gs_last_error(void) { return tl_err.c_str(); }
int32_t gs_version(void) { return GS_ABI_VERSION; }

gs_status gs_set_node_steps(int32_t node_steps) {
    if (node_steps < 0 || node_steps > GS_NODE_STEPS) return fail(GS_ERR_ARG, "node_steps outside [0, GS_NODE_STEPS]");
    g_node_steps = node_steps;
    return GS_OK;
}

gs_status gs_set_camera_batch(int32_t cam_batch) {
    if (cam_batch < 0 || cam_batch > 64) return fail(GS_ERR_ARG, "camera batch outside [0, 64]");
    g_cam_batch = cam_batch;
    return GS_OK;
}

gs_status gs_set_tuning(int32_t shade_batch, int32_t blocks_per_cu, int32_t leaf_batch, int32_t sample_chunk) {
    if (shade_batch < 0 || shade_batch > 64 || blocks_per_cu < 0 || blocks_per_cu > 8 || leaf_batch < 0 ||
        leaf_batch > 64 || sample_chunk < -1)
        return fail(GS_ERR_ARG, "bad tuning");
    g_sample_chunk = sample_chunk;
    g_leaf_batch = leaf_batch;
    g_shade_batch = shade_batch;
    g_blocks_per_cu = blocks_per_cu;
    return GS_OK;
}

gs_status gs_set_placement(int32_t mode) {
    if (mode != 0 && mode != 1) return fail(GS_ERR_ARG, "placement mode is 0 or 1");
    g_placement = mode;
    return GS_OK;
}

gs_status gs_set_adaptive_mode(int32_t mode) {
    if (mode < 0 || mode > 2)
        return fail(GS_ERR_ARG, "adaptive mode is 0 (per-lane loop), 1 (auto) or 2 (batch rounds)");
    g_adaptive_rounds = mode;
    return GS_OK;
}

gs_status gs_debug_set_round_items(int32_t mode) {
    if (mode < -1 || mode > 1) return fail(GS_ERR_ARG, "round item mode is -1 (auto), 0 (split) or 1 (whole)");
    g_round_whole = mode;
    return GS_OK;
}

gs_status gs_debug_set_cube_lists(int32_t on) {
    if (on != 0 && on != 1) return fail(GS_ERR_ARG, "cube lists are 0 (the list loop) or 1 (cube_test)");
    g_cube_lists = on;
    return GS_OK;
}

gs_status gs_debug_set_partial_budget(uint64_t bytes) {
    g_partial_budget.store(bytes ? bytes : (4ull << 30));
    return GS_OK;
}

gs_status gs_debug_set_guided_tail(int32_t fine_chunk, int32_t tail_pct) {
    if (fine_chunk < 0 || tail_pct < 0) return fail(GS_ERR_ARG, "fine_chunk and tail_pct are >= 0 (0: the default)");
    // (the tail's items are single samples, which the combine regroups into the coarse chunks:
    // other sizes would make the association depend on which tiles run in the tail)
    if (fine_chunk > 1) return fail(GS_ERR_ARG, "fine_chunk is 0 or 1 (1-sample tail items)");
    g_tail_pct.store(tail_pct);
    return GS_OK;
}

gs_status gs_device_scene_create(const gs_flat_scene* s, gs_device_scene** out) {
    if (!s || !out) return fail(GS_ERR_ARG, "null argument");
    *out = nullptr;
    uint32_t depth = 1;
    bool nested = false, general = false;
    std::vector<uint8_t> inst_reached, media_reached;
    gs_status v = validate(*s, &depth, &nested, &inst_reached, &general, &media_reached);
    if (v != GS_OK) return v;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(GS_ERR_NO_DEVICE, "no HIP device visible");

    // Quad::cube lists (cube_test): their device list records and cube records.  Their quads
    // are never read through the quad mirror, so the mirror holds a prefix of the quads only
    // as far as the last other quad in it (mirror_quads).
    std::vector<gs_list> dlists(s->lists, s->lists + s->n_lists);
    std::vector<double> cubes;
    std::vector<uint8_t> in_cube(s->n_quads, 0);
    {
        struct Cube {
            uint32_t list, q0;
            double rec[GS_CUBE_DOUBLES];
        };
        std::vector<Cube> found;
        for (uint32_t i = 0; g_cube_lists && i < s->n_lists; i++) {
            Cube c;
            if (!cube_record(*s, s->lists[i], c.q0, c.rec)) continue;
            c.list = i;
            found.push_back(c);
        }
        // (the LDS mirror holds a prefix of the cube records in list order: largest boxes
        // first measured neutral, profiles/r04/ab_cube_order.txt)
        for (const Cube& c : found) {
            dlists[c.list] = gs_list{(uint32_t)(cubes.size() / GS_CUBE_DOUBLES), GS_CUBE_FLAG | c.q0};
            cubes.insert(cubes.end(), c.rec, c.rec + GS_CUBE_DOUBLES);
            for (uint32_t k = 0; k < 6; k++) in_cube[c.q0 + k] = 1;
        }
    }
    // (a quad may also be referenced directly elsewhere: any ref outside a cube list keeps
    // it a mirror candidate -- conservatively, every quad not in a cube list)
    std::vector<uint32_t> single_quads;
    for (uint32_t i = 0; i < s->n_quads; i++)
        if (!in_cube[i]) single_quads.push_back(i);

    std::vector<gs_instance> insts(s->instances, s->instances + s->n_instances);
    std::vector<gs_medium> media(s->media, s->media + s->n_media);
    // The threaded top-level tree (see THR_END): pre-order records of nodes and leaf
    // occurrences; raw links first, then split into node and leaf arrays.
    std::vector<DNode> thr;
    std::vector<uint8_t> thr_leaf;
    std::vector<TNode> tnodes;
    std::vector<TBox> tboxes;
    std::vector<TLeaf> tleaves;
    uint32_t lds_nodes = 0, lds_leaves = 0, lds_quads = 0, lds_cubes = 0, thr_root_tagged = THR_END;
    ThreadedTree tree_keep;  // kept by the scene: re-placed after a launch's pilot (place_records)
    std::vector<uint32_t> nroot_rec_keep, nroots_placed;  // the nested trees' root records, their links
    std::vector<uint32_t> placed_pos;
    double nodes_per_leaf = 0.0, other_leaf_frac = 0.0;
    bool leaf_runs = false, sph_leaves = false;
    int32_t auto_node_steps = GS_NODE_STEPS;
    {
        // Iterative pre-order: a node pushes a "close" marker below its children, which
        // sets its miss link once its subtree is emitted.
        std::vector<std::pair<uint32_t, bool>> work{{s->root, false}};
        while (!work.empty()) {
            auto [x, close] = work.back();
            work.pop_back();
            if (close) {  // x = record index of a node whose subtree is now complete
                thr[x].right = (uint32_t)thr.size();
                continue;
            }
            const uint32_t idx = (uint32_t)thr.size();
            DNode rec{};
            if ((x >> GS_REF_SHIFT) == GS_REF_NODE) {
                const gs_node& n = s->nodes[x & GS_REF_MASK];
                rec = DNode{n.min[0], n.min[1], n.min[2], n.max[0], n.max[1], n.max[2], idx + 1u, 0u, 0u, 0u};
                thr.push_back(rec);
                thr_leaf.push_back(0);
                work.push_back({idx, true});
                if (n.right != GS_REF_NONE) work.push_back({n.right, false});
                work.push_back({n.left, false});
            } else {
                if ((x >> GS_REF_SHIFT) == GS_REF_SPHERE) {
                    const gs_sphere& q = s->spheres[x & GS_REF_MASK];
                    rec.mnx = q.center[0];
                    rec.mny = q.center[1];
                    rec.mnz = q.center[2];
                    rec.mxx = q.radius;
                }
                rec.left = idx + 1u;  // next
                rec.right = x;  // the primitive's ref
                thr.push_back(rec);
                thr_leaf.push_back(1);
            }
        }
        const uint32_t n = (uint32_t)thr.size();
        // (the top-level walk's end: RAW_END, so records appended below keep their indices)
        for (uint32_t i = 0; i < n; i++) {
            if (thr[i].left >= n) thr[i].left = RAW_END;
            if (!thr_leaf[i] && thr[i].right >= n) thr[i].right = RAW_END;
        }
        // Placement: the records a ray is most likely to test first, so a block can mirror
        // them in LDS; the rest in pre-order.  Static estimate (until a launch's pilot
        // measures the real visits, place_records): the smallest surface area of a box on
        // the record's path from the root (a ray tests a record only if it hit all of
        // them), ties broken by depth.  Links are explicit, so placement does not change
        // the walk.
        std::vector<uint32_t> depth(n, 0);
        std::vector<double> score(n, 0.0);
        {
            for (uint32_t i = 0; i < n; i++)
                if (!thr_leaf[i]) {
                    // records are pre-order: a node's descendants follow it, so depths
                    // propagate in one forward pass
                    for (uint32_t c = thr[i].left; c < thr[i].right && c < n;) {
                        depth[c] = depth[i] + 1;
                        c = thr_leaf[c] ? c + 1 : thr[c].right;  // next child of node i
                    }
                }
            // score = surface area of the parent's box (the chance a ray tests the record)
            if (n) score[0] = 1e308;
            for (uint32_t i = 0; i < n; i++)
                if (!thr_leaf[i]) {
                    const DNode& b = thr[i];
                    const double dx = b.mxx - b.mnx, dy = b.mxy - b.mny, dz = b.mxz - b.mnz;
                    const double sa = dx * dy + dy * dz + dz * dx;
                    for (uint32_t c = thr[i].left; c < thr[i].right && c < n;) {
                        score[c] = std::min(score[i], sa);
                        c = thr_leaf[c] ? c + 1 : thr[c].right;
                    }
                }
            // Expected node tests per leaf test (the score over the root box's area is the
            // chance a ray entering the root tests the record).
            if (n && !thr_leaf[0]) {
                const DNode& b = thr[0];
                const double dx = b.mxx - b.mnx, dy = b.mxy - b.mny, dz = b.mxz - b.mnz;
                const double sa_root = dx * dy + dy * dz + dz * dx;
                double pn = 0.0, pl = 0.0, po = 0.0;
                for (uint32_t i = 0; i < n; i++) {
                    const double p = i == 0 ? 1.0 : (sa_root > 0.0 ? std::min(1.0, score[i] / sa_root) : 1.0);
                    (thr_leaf[i] ? pl : pn) += p;
                    if (thr_leaf[i] && (thr[i].right >> GS_REF_SHIFT) != GS_REF_SPHERE) po += p;
                }
                nodes_per_leaf = pl > 0.0 ? pn / pl : 0.0;
                other_leaf_frac = pl > 0.0 ? po / pl : 0.0;
            } else if (n) {
                other_leaf_frac = (thr[0].right >> GS_REF_SHIFT) != GS_REF_SPHERE ? 1.0 : 0.0;
            }
        }
        // BVHs under instance chains (GS_FEAT_NESTED: final_scene's box of balls, main.rs:
        // 741-755): each distinct tree under a reached instance is threaded once, in pre-order,
        // into the same records after the top-level tree -- node {box, hit = next record, miss
        // = after its subtree}, leaf {a stationary sphere inline, next, ABI ref} -- its last
        // links RAW_RET (THR_RET: back to the top-level ray); the instance's device child
        // becomes GS_REF_NODE | tree index, and nroot_rec[tree] its root record.  The lane
        // walks it in the main loop's node and leaf passes (render kernel, leaf pass), so its
        // records are placed and mirrored with the top level's by measured visits.
        {
            std::unordered_map<uint32_t, uint32_t> tree_of;  // gs node index -> tree
            std::vector<double> tree_score;                   // a tree's best entry (its leaves' score)
            std::vector<uint32_t> tree_depth;
            // thread the tree at BVH node ref `node_ref` once; returns its tree index
            auto thread_tree = [&](uint32_t node_ref) -> uint32_t {
                const uint32_t root = node_ref & GS_REF_MASK;
                auto it = tree_of.find(root);
                if (it != tree_of.end()) return it->second;
                const uint32_t first = (uint32_t)thr.size();
                struct Work {
                    uint32_t x;
                    bool close;
                };
                std::vector<Work> work{{node_ref, false}};
                while (!work.empty()) {
                    const Work w = work.back();
                    work.pop_back();
                    if (w.close) {
                        thr[w.x].right = (uint32_t)thr.size();
                        continue;
                    }
                    const uint32_t idx = (uint32_t)thr.size();
                    DNode rec{};
                    if ((w.x >> GS_REF_SHIFT) == GS_REF_NODE) {
                        const gs_node& nd = s->nodes[w.x & GS_REF_MASK];
                        rec = DNode{nd.min[0], nd.min[1], nd.min[2], nd.max[0], nd.max[1], nd.max[2], idx + 1u, 0u, 0u, 0u};
                        thr.push_back(rec);
                        thr_leaf.push_back(0);
                        work.push_back({idx, true});
                        if (nd.right != GS_REF_NONE) work.push_back({nd.right, false});
                        work.push_back({nd.left, false});
                    } else {
                        if ((w.x >> GS_REF_SHIFT) == GS_REF_SPHERE) {
                            const gs_sphere& q = s->spheres[w.x & GS_REF_MASK];
                            rec.mnx = q.center[0];
                            rec.mny = q.center[1];
                            rec.mnz = q.center[2];
                            rec.mxx = q.radius;
                        }
                        rec.left = idx + 1u;
                        rec.right = w.x;
                        thr.push_back(rec);
                        thr_leaf.push_back(1);
                    }
                }
                const uint32_t end = (uint32_t)thr.size();
                for (uint32_t k = first; k < end; k++) {
                    if (thr[k].left == end) thr[k].left = RAW_RET;
                    if (!thr_leaf[k] && thr[k].right == end) thr[k].right = RAW_RET;
                }
                const uint32_t tr = (uint32_t)nroot_rec_keep.size();
                tree_of.emplace(root, tr);
                nroot_rec_keep.push_back(first);
                tree_score.push_back(0.0);
                tree_depth.push_back(0);
                return tr;
            };
            for (size_t ii = 0; ii < insts.size(); ii++) {
                gs_instance& in = insts[ii];
                if ((in.child >> GS_REF_SHIFT) != GS_REF_NODE) continue;
                // Only instances a reachable leaf walks: validate() checked their trees (indices,
                // depth, leaves); an unreachable one is never read by the kernel and may be
                // malformed, so its node child is dropped, not walked.
                if (!inst_reached[ii]) {
                    in.child = GS_REF_NONE;
                    continue;
                }
                in.child = GS_MAKE_REF(GS_REF_NODE, thread_tree(in.child));
            }
            // (GS_FEAT_GENERAL) a BVH that is a medium's boundary with no chain: threaded alike,
            // the medium's device boundary the tree's ref (tree_test)
            if (general)
                for (size_t mi = 0; mi < media.size(); mi++)
                    if (media_reached[mi] && (media[mi].boundary >> GS_REF_SHIFT) == GS_REF_NODE)
                        media[mi].boundary = GS_MAKE_REF(GS_REF_NODE, thread_tree(media[mi].boundary));
            if (nroot_rec_keep.size() > GS_REF_MASK) return fail(GS_ERR_UNSUPPORTED, "too many BVHs under instances");
            // Static estimate for the nested records: a top-level leaf whose chain ends in a
            // tree gives it its score and depth; inside, the smallest surface area on the path
            // relative to the tree's root box (rigid transforms keep areas).
            for (uint32_t i = 0; i < n; i++) {
                if (!thr_leaf[i]) continue;
                uint32_t r = thr[i].right;
                for (int k = 0; k < GS_MAX_CHAIN && (r >> GS_REF_SHIFT) == GS_REF_INSTANCE; k++) r = insts[r & GS_REF_MASK].child;
                if ((r >> GS_REF_SHIFT) != GS_REF_NODE) continue;
                const uint32_t tr = r & GS_REF_MASK;
                if (score[i] > tree_score[tr]) {
                    tree_score[tr] = score[i];
                    tree_depth[tr] = depth[i] + 1;
                }
            }
            const uint32_t total = (uint32_t)thr.size();
            depth.resize(total, 0);
            score.resize(total, 0.0);
            for (size_t tr = 0; tr < nroot_rec_keep.size(); tr++) {
                const uint32_t first = nroot_rec_keep[tr];
                const uint32_t end = tr + 1 < nroot_rec_keep.size() ? nroot_rec_keep[tr + 1] : total;
                const DNode& rb = thr[first];
                const double rdx = rb.mxx - rb.mnx, rdy = rb.mxy - rb.mny, rdz = rb.mxz - rb.mnz;
                const double sa_root = rdx * rdy + rdy * rdz + rdz * rdx;
                depth[first] = tree_depth[tr];
                score[first] = tree_score[tr];
                std::vector<double> local(end - first, sa_root);
                for (uint32_t i = first; i < end; i++)
                    if (!thr_leaf[i]) {
                        const DNode& b = thr[i];
                        const double dx = b.mxx - b.mnx, dy = b.mxy - b.mny, dz = b.mxz - b.mnz;
                        const double sa = std::min(local[i - first], dx * dy + dy * dz + dz * dx);
                        for (uint32_t c = thr[i].left; c < thr[i].right && c < end;) {
                            depth[c] = depth[i] + 1;
                            local[c - first] = sa;
                            score[c] = sa_root > 0.0 ? tree_score[tr] * std::min(1.0, sa / sa_root) : tree_score[tr];
                            c = thr_leaf[c] ? c + 1 : thr[c].right;
                        }
                    }
            }
        }
        tree_keep = ThreadedTree{thr, thr_leaf, std::move(depth), std::move(score)};
        const Placed pl = place_records(tree_keep, nullptr, single_quads,
                                        g_lds_mirror < 0 ? lds_mirror_budget() : g_lds_mirror, nroot_rec_keep,
                                        (uint32_t)(cubes.size() / GS_CUBE_DOUBLES));
        nroots_placed = pl.nroots;
        tnodes = pl.tnodes;
        tboxes = pl.tboxes;
        tleaves = pl.tleaves;
        lds_nodes = pl.lds_nodes;
        lds_leaves = pl.lds_leaves;
        lds_quads = pl.lds_quads;
        lds_cubes = pl.lds_cubes;
        thr_root_tagged = pl.root;
        placed_pos = pl.pos;
        // Leaf runs pay when at least a quarter of the leaf records are the first of two
        // adjacent sphere leaves (C4's two-sphere leaves of BVH.rs:44-55: ~half).
        {
            auto is_sph = [&](uint32_t i) { return thr_leaf[i] && (thr[i].right >> GS_REF_SHIFT) == GS_REF_SPHERE; };
            // (over every record: a nested tree's leaf pairs run in the same leaf passes)
            const uint32_t na = (uint32_t)thr.size();
            uint64_t leaves = 0, pairs = 0;
            for (uint32_t i = 0; i < na; i++) {
                leaves += thr_leaf[i];
                pairs += i + 1 < na && is_sph(i) && is_sph(i + 1) && thr[i].left == i + 1;
            }
            leaf_runs = leaves && pairs * 4 >= leaves;
            sph_leaves = leaves > 0;
            for (uint32_t i = 0; i < n && sph_leaves; i++) sph_leaves = !thr_leaf[i] || is_sph(i);
            // Node steps per node pass (MI355X, Msamples/s).  Sphere-only trees take long
            // node runs (C4: 3 -> 6101, 8 -> 6347).  Trees whose leaf tests are mostly other
            // kinds keep their lanes in step, one node per pass, so that a leaf pass finds
            // them at one leaf and takes the scalar-load path (C3: 1 -> 10336, 3 -> 9194,
            // 8 -> 6818).  Mixed trees in between (C5: 3 -> 5629, 8 -> 5088).
            auto_node_steps = other_leaf_frac == 0.0 ? GS_NODE_STEPS : (other_leaf_frac >= 0.5 ? 1 : 3);
        }
    }
    if (tnodes.size() >= (1u << 26) || tleaves.size() >= (1u << 26))
        return fail(GS_ERR_UNSUPPORTED, "more than 2^26 top-level BVH records");
    bool cert_boxes = true;
    for (const TBox& b : tboxes)
        for (double v : {b.mnx, b.mny, b.mnz, b.mxx, b.mxy, b.mxz})
            if (!(std::fabs(v) <= 1e15)) cert_boxes = false;
    std::vector<TQuad> tquads(s->n_quads);
    for (uint32_t i = 0; i < s->n_quads; i++) {
        const gs_quad& q = s->quads[i];
        tquads[i] = TQuad{q.normal[0], q.normal[1], q.normal[2], q.d, q.q[0], q.q[1], q.q[2], q.u[0],
                          q.u[1],      q.u[2],      q.v[0],      q.v[1], q.v[2], q.w[0], q.w[1], q.w[2]};
    }
    std::vector<DSphere> sph(s->n_spheres);
    std::vector<uint32_t> sph_mat(s->n_spheres);
    for (uint32_t i = 0; i < s->n_spheres; i++) {
        const gs_sphere& x = s->spheres[i];
        sph[i] = DSphere{x.center[0], x.center[1], x.center[2], x.radius};
        sph_mat[i] = x.material;
    }
    std::vector<DMaterial> mats(s->n_materials);
    for (uint32_t i = 0; i < s->n_materials; i++) {
        const gs_material& m = s->materials[i];
        DMaterial d{};
        d.texture = m.texture;
        const bool textured = m.kind == GS_MAT_LAMBERTIAN || m.kind == GS_MAT_DIFFUSE_LIGHT || m.kind == GS_MAT_ISOTROPIC;
        d.needs_uv = textured ? tex_needs_uv(*s, m.texture) : 0;
        if (textured) {
            const gs_texture& t = s->textures[m.texture];
            const bool solid = t.kind == GS_TEX_SOLID;
            const bool checker2 = t.kind == GS_TEX_CHECKERED && s->textures[t.even].kind == GS_TEX_SOLID &&
                                  s->textures[t.odd].kind == GS_TEX_SOLID;
            if (m.kind == GS_MAT_LAMBERTIAN) {
                d.kind = solid ? DM_LAMB_SOLID : (checker2 ? DM_LAMB_CHECKER : DM_LAMB_TEX);
            } else if (m.kind == GS_MAT_ISOTROPIC) {
                d.kind = solid ? DM_ISO_SOLID : DM_ISO_TEX;
            } else {
                d.kind = solid ? DM_LIGHT_SOLID : DM_LIGHT_TEX;
            }
            if (solid) {
                for (int k = 0; k < 3; k++) d.a[k] = t.color[k];
            } else if (checker2 && m.kind == GS_MAT_LAMBERTIAN) {
                for (int k = 0; k < 3; k++) {
                    d.a[k] = s->textures[t.even].color[k];
                    d.b[k] = s->textures[t.odd].color[k];
                }
                d.param = t.scale_inv;
            }
        } else if (m.kind == GS_MAT_METAL) {
            d.kind = DM_METAL;
            for (int k = 0; k < 3; k++) d.a[k] = m.albedo[k];
            d.param = m.param;
        } else {
            d.kind = DM_DIELECTRIC;
            d.param = m.param;
        }
        mats[i] = d;
    }
    // HDRI: keep 4-byte RGBE texels when every f32 texel round-trips exactly.
    std::vector<uint32_t> rgbe;
    if (s->background.kind == GS_BG_HDRI) {
        const uint64_t n = (uint64_t)s->background.width * s->background.height;
        rgbe.resize(n);
        for (uint64_t k = 0; k < n && !rgbe.empty(); k++)
            if (!encode_rgbe(s->hdri_rgb + 3 * k, &rgbe[k])) rgbe.clear();
    }
    Layout L;
    size_t o_nroots = L.add(nroots_placed.data(), nroots_placed.size() * 4);
    size_t o_tnodes = L.add(tnodes.data(), tnodes.size() * sizeof(TNode));
    size_t o_tboxes = L.add(tboxes.data(), tboxes.size() * sizeof(TBox));
    size_t o_tleaves = L.add(tleaves.data(), tleaves.size() * sizeof(TLeaf));
    size_t o_tquads = L.add(tquads.data(), tquads.size() * sizeof(TQuad));
    size_t o_sph = L.add(sph.data(), sph.size() * sizeof(DSphere));
    size_t o_sphm = L.add(sph_mat.data(), sph_mat.size() * 4);
    size_t o_msph = L.add(s->mspheres, s->n_mspheres * sizeof(gs_msphere));
    size_t o_quad = L.add(s->quads, s->n_quads * sizeof(gs_quad));
    size_t o_tri = L.add(s->triangles, s->n_triangles * sizeof(gs_triangle));
    size_t o_list = L.add(dlists.data(), dlists.size() * sizeof(gs_list));
    size_t o_cubes = L.add(cubes.data(), cubes.size() * sizeof(double));
    size_t o_lref = L.add(s->list_refs, s->n_list_refs * 4);
    size_t o_inst = L.add(insts.data(), insts.size() * sizeof(gs_instance));
    size_t o_media = L.add(media.data(), media.size() * sizeof(gs_medium));
    size_t o_perm = L.add(s->noise_perm, s->noise_perm ? s->n_noise_perm : 0);
    size_t o_mat = L.add(mats.data(), mats.size() * sizeof(DMaterial));
    size_t o_tex = L.add(s->textures, s->n_textures * sizeof(gs_texture));
    size_t o_img = L.add(s->images, s->n_images * sizeof(gs_image));
    size_t o_texel = L.add(s->texels8, s->n_texels8);
    size_t o_hdri = L.add(s->hdri_rgb, (s->background.kind == GS_BG_HDRI && rgbe.empty()) ? s->n_hdri_floats * 4 : 0);
    size_t o_rgbe = L.add(rgbe.data(), rgbe.size() * 4);
    size_t o_slot[kLaunchSlots];
    for (int k = 0; k < kLaunchSlots; k++) o_slot[k] = L.add(nullptr, 256 + sizeof(KParams));  // queue, params

    auto ds = new gs_device_scene();
    (void)hipGetDevice(&ds->device);
    ds->bytes = L.blob.size();
    if (hipMalloc(&ds->mem, ds->bytes) != hipSuccess) {
        delete ds;
        return fail(GS_ERR_OOM, "hipMalloc of " + std::to_string(L.blob.size()) + " bytes failed");
    }
    hipError_t e = hipMemcpy(ds->mem, L.blob.data(), ds->bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(ds->mem);
        delete ds;
        return fail(GS_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
    }
    uint8_t* b = (uint8_t*)ds->mem;
    DevScene& d = ds->dev;
    d.nroots = (const uint32_t*)(b + o_nroots);
    d.spheres = (const DSphere*)(b + o_sph);
    d.sphere_mat = (const uint32_t*)(b + o_sphm);
    d.mspheres = (const gs_msphere*)(b + o_msph);
    d.quads = (const gs_quad*)(b + o_quad);
    d.tris = (const gs_triangle*)(b + o_tri);
    d.lists = (const gs_list*)(b + o_list);
    d.list_refs = (const uint32_t*)(b + o_lref);
    d.cubes = (const double*)(b + o_cubes);
    d.inst = (const gs_instance*)(b + o_inst);
    d.media = (const gs_medium*)(b + o_media);
    d.noise_perm = (const uint8_t*)(b + o_perm);
    d.mats = (const DMaterial*)(b + o_mat);
    d.texs = (const gs_texture*)(b + o_tex);
    d.images = (const gs_image*)(b + o_img);
    d.texels = (const uint8_t*)(b + o_texel);
    d.hdri = (const float*)(b + o_hdri);
    d.hdri_rgbe = rgbe.empty() ? nullptr : (const uint32_t*)(b + o_rgbe);
    d.bg = s->background;
    d.root = device_ref(s->root);
    d.tnodes = (const TNode*)(b + o_tnodes);
    d.tboxes = (const TBox*)(b + o_tboxes);
    d.tleaves = (const TLeaf*)(b + o_tleaves);
    for (int k = 0; k < kLaunchSlots; k++) {
        ds->slots[k].queue = (uint32_t*)(b + o_slot[k]);
        ds->slots[k].params = (KParams*)(b + o_slot[k] + 256);
        if (hipEventCreateWithFlags(&ds->slots[k].done, hipEventDisableTiming) != hipSuccess) {
            gs_device_scene_destroy(ds);
            return fail(GS_ERR_HIP, "hipEventCreateWithFlags failed");
        }
    }
    ds->n_nodes = s->n_nodes;
    ds->tnodes = (const TNode*)(b + o_tnodes);
    ds->tboxes = (const TBox*)(b + o_tboxes);
    ds->tleaves = (const TLeaf*)(b + o_tleaves);
    ds->tquads = (const TQuad*)(b + o_tquads);
    ds->thr_root = thr_root_tagged;
    ds->lds_nodes = lds_nodes;
    ds->lds_leaves = lds_leaves;
    ds->lds_quads = lds_quads;
    ds->nroot_rec = nroot_rec_keep;
    ds->nroots = (uint32_t*)(b + o_nroots);
    ds->single_quads = single_quads;
    ds->lds_cubes = lds_cubes;
    ds->n_cubes = (uint32_t)(cubes.size() / GS_CUBE_DOUBLES);
    ds->node_records = (uint32_t)tnodes.size();
    ds->leaf_records = (uint32_t)tleaves.size();
    ds->nodes_per_leaf = nodes_per_leaf;
    ds->other_leaf_frac = other_leaf_frac;
    ds->bvh_depth = depth < 1 ? 1 : depth;
    ds->feat = (s->n_media != 0 ? GS_FEAT_MEDIA : 0) | (nested ? GS_FEAT_NESTED : 0) | (leaf_runs ? GS_FEAT_LEAFRUN : 0);
    if (!(ds->feat & (GS_FEAT_MEDIA | GS_FEAT_NESTED)) && lds_nodes == tnodes.size() && lds_leaves == tleaves.size())
        ds->feat |= GS_FEAT_LDSTREE;  // (cleared at launch if the device's LDS cannot hold it all)
    {  // staged shading when three or more of its sharing cases can meet in one wave
        bool lamb = false, metal = false, diel = false, iso = false;
        for (const DMaterial& m : mats) {
            lamb |= m.kind >= DM_LAMB_SOLID && m.kind <= DM_LAMB_TEX;
            metal |= m.kind == DM_METAL;
            diel |= m.kind == DM_DIELECTRIC;
            iso |= m.kind == DM_ISO_SOLID || m.kind == DM_ISO_TEX;
        }
        const int cases = (int)lamb + (int)metal + (int)diel + (int)iso + (int)(s->background.kind != GS_BG_SOLID);
        if (cases >= 3 && !(ds->feat & (GS_FEAT_MEDIA | GS_FEAT_NESTED))) ds->feat |= GS_FEAT_MIXED;
    }
    // (round 6: also without leaf runs -- C1, C2, A1's lone sphere -- for the sphere-only hit record)
    if (sph_leaves && !(ds->feat & (GS_FEAT_MEDIA | GS_FEAT_NESTED))) ds->feat |= GS_FEAT_SPHLEAF;
    if ((ds->feat & (GS_FEAT_SPHLEAF | GS_FEAT_MIXED)) == (GS_FEAT_SPHLEAF | GS_FEAT_MIXED) && g_plain_kernels) {
        // every hit a stationary sphere (SPHLEAF): plain materials, no uv -> GS_FEAT_PLAIN
        bool plain = true;
        for (const DMaterial& m : mats)
            plain &= (m.kind == DM_LAMB_SOLID || m.kind == DM_LAMB_CHECKER || m.kind == DM_METAL ||
                      m.kind == DM_DIELECTRIC) && !m.needs_uv;
        if (plain) ds->feat |= GS_FEAT_PLAIN;
    }
    // compositions only the catch-all instantiation walks (round 6; validate)
    if (general) ds->feat = GS_FEAT_GENERAL_KERNEL;
    ds->cert_boxes = cert_boxes;
    ds->node_steps = auto_node_steps;
    // Scenes with BVHs under instances (kind-batched leaf passes over many leaf kinds) gather
    // more lanes per leaf pass, each pass serving one kind, and step nodes in full passes:
    // final_scene 1440^2 x 64 spp, (leaf batch, node steps): (12, 1) 1206, (32, 3) 1540,
    // (48, 3) 1594, (48, 8) 1679, (64, 8) 1662 Msamples/s (profiles/r03/sweep_final_scene_
    // leaf_batch*.txt).  Not for staged shading alone: C5 leaf batch 12 6178, 24 5989, 48 5236.
    // ... and shade smaller batches (round 4, after the nested-leaf changes; shade batch x leaf
    // batch at 8 node steps, twice: 44 / 48: 2 396, 2 462; 44 / 56: 2 449, 2 453; 52 / 48:
    // 2 365, 2 398 Msamples/s, profiles/r04/sweep_final_scene_shade_leaf_batch.txt).
    // Round 5 walks the nested BVHs in the main node passes, so a leaf pass holds fewer
    // leaf kinds and smaller batches pay: leaf batch 48 -> 2 577, 24 -> 2 644-2 660
    // Msamples/s (profiles/r05).
    if (ds->feat & GS_FEAT_NESTED) {
        ds->leaf_batch = GS_KIND_LEAF_BATCH;
        ds->shade_batch = GS_KIND_SHADE_BATCH;
        ds->node_steps = std::max<int32_t>(ds->node_steps, GS_KIND_NODE_STEPS);
    }
    ds->tree = std::move(tree_keep);
    ds->pos = std::move(placed_pos);
    ds->n_quads = s->n_quads;
    ds->mirror_budget = g_lds_mirror < 0 ? lds_mirror_budget() : g_lds_mirror;
    *out = ds;
    return GS_OK;
}

gs_status gs_device_scene_info(const gs_device_scene* ds, gs_scene_info* out) {
    if (!ds || !out) return fail(GS_ERR_ARG, "null argument");
    gs_scene_info i{};
    i.node_records = ds->node_records;
    i.leaf_records = ds->leaf_records;
    i.lds_nodes = ds->lds_nodes;
    i.lds_leaves = ds->lds_leaves;
    i.lds_quads = ds->lds_quads;
    i.feat = ds->feat;
    const int32_t t_steps = g_node_steps.load(std::memory_order_relaxed);
    i.node_steps = std::max(1, std::min<int32_t>(unroll_steps(ds->feat), t_steps > 0 ? t_steps : ds->node_steps));
    i.cert_boxes = ds->cert_boxes ? 1 : 0;
    i.nodes_per_leaf = ds->nodes_per_leaf;
    i.other_leaf_frac = ds->other_leaf_frac;
    i.placement = ds->placement.load(std::memory_order_acquire);
    i.long_samples = ds->long_samples.load(std::memory_order_relaxed) ? 1 : 0;
    i.pilot_ms = ds->pilot_ms;
    *out = i;
    return GS_OK;
}

gs_status gs_device_scene_destroy(gs_device_scene* ds) {
    if (!ds) return GS_OK;
    for (auto& sl : ds->slots) {
        if (sl.done) {
            if (sl.used) (void)hipEventSynchronize(sl.done);
            (void)hipEventDestroy(sl.done);
        }
        if (sl.partial) (void)hipFree(sl.partial);
        if (sl.rbuf) (void)hipFree(sl.rbuf);
        if (sl.nest_save) (void)hipFree(sl.nest_save);
    }
    if (ds->mem) (void)hipFree(ds->mem);
    delete ds;
    return GS_OK;
}

#ifndef GS_SHORT_SAMPLE_LANE_US
#define GS_SHORT_SAMPLE_LANE_US 50.0
#endif
// Compute units of a device (cached: the attribute query costs ~0.5 ms).
static int device_cus(int dev) {
    static std::atomic<int> cache[64];
    if (dev < 0 || dev >= 64) return 256;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (v == 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

void gs_device_scene_note_frame(gs_device_scene* ds, double kernel_ms, uint64_t samples) {
    if (!ds || !(kernel_ms > 0.0) || samples == 0) return;
    const double lanes = (double)device_cus(ds->device) * GS_BLOCK;
    const double lus = kernel_ms * 1e3 * lanes / (double)samples;
    ds->lane_us_per_sample.store(lus, std::memory_order_relaxed);
    if (lus > GS_SHORT_SAMPLE_LANE_US) ds->long_samples.store(true, std::memory_order_relaxed);
}

static bool part_ok(const gs_camera* cam, const gs_partition* p) {
    return cam && p && cam->image_width > 0 && cam->image_height > 0 && p->world_size >= 1 && p->rank >= 0 &&
           p->rank < p->world_size && p->tile_w > 0 && p->tile_h > 0 && (int64_t)p->tile_w * p->tile_h <= (1 << 20) &&
           (!p->d_tile_order || p->slots_per_rank > 0);
}

int64_t gs_partition_capacity(const gs_camera* cam, const gs_partition* p) {
    if (!part_ok(cam, p)) return -1;
    if (p->d_tile_order) return (int64_t)p->slots_per_rank * p->tile_w * p->tile_h;
    int64_t tx = (cam->image_width + p->tile_w - 1) / p->tile_w;
    int64_t ty = (cam->image_height + p->tile_h - 1) / p->tile_h;
    int64_t nt = tx * ty;
    int64_t mine = nt > p->rank ? (nt - p->rank + p->world_size - 1) / p->world_size : 0;
    return mine * p->tile_w * p->tile_h;
}

static void (*kernel_for(int feat))(KArgs) {
#ifdef GS_ONLY_FEAT  // register-pressure experiments (tools/resource_usage.sh): one instantiation
    (void)feat;
    return gs_render_kernel<GS_ONLY_FEAT>;
#else
    // The product instantiations, each also in its fixed-spp form (| GS_FEAT_FIXED); those
    // without media or BVHs under instances also in the split batch-round form (| GS_FEAT_FIXED
    // | GS_FEAT_RSPLIT; has_rsplit).
#define GS_K(F)                                              \
    case (F): return gs_render_kernel<(F)>;                  \
    case (F) | GS_FEAT_FIXED: return gs_render_kernel<(F) | GS_FEAT_FIXED>;
#define GS_KR(F) \
    GS_K(F)      \
    case (F) | GS_FEAT_FIXED | GS_FEAT_RSPLIT: return gs_render_kernel<(F) | GS_FEAT_FIXED | GS_FEAT_RSPLIT>;
    switch (feat) {
        GS_K(GS_FEAT_MEDIA)
        GS_K(GS_FEAT_NESTED)
        GS_K(GS_FEAT_MEDIA | GS_FEAT_NESTED)
        GS_KR(GS_FEAT_LEAFRUN)
        GS_K(GS_FEAT_LEAFRUN | GS_FEAT_MEDIA)
        GS_K(GS_FEAT_LEAFRUN | GS_FEAT_NESTED)
        GS_K(GS_FEAT_LEAFRUN | GS_FEAT_MEDIA | GS_FEAT_NESTED)
        GS_KR(GS_FEAT_LDSTREE)
        GS_KR(GS_FEAT_LDSTREE | GS_FEAT_LEAFRUN)
        GS_KR(GS_FEAT_MIXED)
        GS_KR(GS_FEAT_MIXED | GS_FEAT_LEAFRUN)
        GS_KR(GS_FEAT_MIXED | GS_FEAT_LDSTREE)
        GS_KR(GS_FEAT_MIXED | GS_FEAT_LDSTREE | GS_FEAT_LEAFRUN)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LEAFRUN)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LEAFRUN | GS_FEAT_LDSTREE)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LEAFRUN | GS_FEAT_MIXED)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LEAFRUN | GS_FEAT_MIXED | GS_FEAT_LDSTREE)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LEAFRUN | GS_FEAT_MIXED | GS_FEAT_PLAIN)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LEAFRUN | GS_FEAT_MIXED | GS_FEAT_PLAIN | GS_FEAT_LDSTREE)
        GS_K(GS_FEAT_GENERAL_KERNEL)
        GS_KR(GS_FEAT_SPHLEAF)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_LDSTREE)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_MIXED)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_MIXED | GS_FEAT_LDSTREE)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_MIXED | GS_FEAT_PLAIN)
        GS_KR(GS_FEAT_SPHLEAF | GS_FEAT_MIXED | GS_FEAT_PLAIN | GS_FEAT_LDSTREE)
        case GS_FEAT_FIXED: return gs_render_kernel<GS_FEAT_FIXED>;
        case GS_FEAT_FIXED | GS_FEAT_RSPLIT: return gs_render_kernel<GS_FEAT_FIXED | GS_FEAT_RSPLIT>;
        case GS_FEAT_PILOT: return gs_render_kernel<GS_FEAT_PILOT>;
        default: return gs_render_kernel<0>;
    }
#undef GS_KR
#undef GS_K
#endif
}
// A split batch round may take the (F | FIXED | RSPLIT) instantiation (kernel_for's GS_KR list).
static bool has_rsplit(int feat) {
#ifdef GS_ONLY_FEAT
    (void)feat;
    return false;
#else
    return (feat & (GS_FEAT_MEDIA | GS_FEAT_NESTED | GS_FEAT_GENERAL | GS_FEAT_VISITS)) == 0;
#endif
}

gs_status gs_render_tiles_async(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                uint64_t seed, const gs_partition* part, float* d_out, gs_counters* d_counters,
                                void* stream) {
    if (!d_out) return fail(GS_ERR_ARG, "null argument");
    gs_render_outputs o{d_out, nullptr, nullptr};
    return gs_render_tiles_ex_async(ds, cam, ss, seed, part, &o, d_counters, stream);
}

gs_status gs_render_tiles_debug_async(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                      uint64_t seed, const gs_partition* part, float* d_out,
                                      gs_counters* d_counters, uint32_t* d_item_visits, void* stream) {
    if (!d_out) return fail(GS_ERR_ARG, "null argument");
    gs_render_outputs o{d_out, nullptr, d_item_visits};
    return gs_render_tiles_ex_async(ds, cam, ss, seed, part, &o, d_counters, stream);
}

gs_status gs_render_tiles_ex_async(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                   uint64_t seed, const gs_partition* part, const gs_render_outputs* outs,
                                   gs_counters* d_counters, void* stream) {
    return gs_render_tiles_timed_async(ds, cam, ss, seed, part, outs, d_counters, stream, nullptr, nullptr);
}

}  // extern "C"

// The launch behind gs_render_tiles_ex_async; k_begin / k_end (nullable, timing events of
// the stream's device) are recorded right around the megakernel, so a caller can time the
// dominant kernel alone (csrc/host/internal.hpp; the frame context's gs_stats.kernel_ms).
// A GS_FEAT_VISITS launch's count buffer: node record positions, then leaf positions.
struct VisitArgs {
    uint32_t* visits;
    uint32_t leaf_base;
};
static gs_status launch(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                        const gs_partition* part, const gs_render_outputs* outs, gs_counters* d_counters, void* stream,
                        hipEvent_t k_begin, hipEvent_t k_end, const VisitArgs* va, bool direct = false,
                        bool zero_counters = false);
static gs_status ensure_placement(gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                  void* stream);

gs_status gs_render_tiles_timed_async(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                      uint64_t seed, const gs_partition* part, const gs_render_outputs* outs,
                                      gs_counters* d_counters, void* stream, hipEvent_t k_begin, hipEvent_t k_end,
                                      bool direct, bool zero_counters) {
    if (!ds || !cam) return fail(GS_ERR_ARG, "null argument");
    gs_status e = ensure_placement(const_cast<gs_device_scene*>(ds), cam, ss, stream);
    if (e != GS_OK) return e;
    return launch(ds, cam, ss, seed, part, outs, d_counters, stream, k_begin, k_end, nullptr, direct, zero_counters);
}

static gs_status launch(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss, uint64_t seed,
                        const gs_partition* part, const gs_render_outputs* outs, gs_counters* d_counters, void* stream,
                        hipEvent_t k_begin, hipEvent_t k_end, const VisitArgs* va, bool direct, bool zero_counters) {
    if (!ds || !cam || !ss || !part || !outs || (!outs->rgb && !outs->rgb8)) return fail(GS_ERR_ARG, "null argument");
    if (!part_ok(cam, part)) return fail(GS_ERR_ARG, "bad partition / image size");
    if (ss->batch_size == 0) return fail(GS_ERR_ARG, "batch_size 0 never terminates (camera.rs:137)");
    int64_t cap = gs_partition_capacity(cam, part);
    if (cap <= 0) {  // nothing to render; a frame context's counters still start from zero
        if (zero_counters && d_counters) HIPCHK(hipMemsetAsync(d_counters, 0, sizeof(gs_counters), (hipStream_t)stream));
        if (k_begin) HIPCHK(hipEventRecord(k_begin, (hipStream_t)stream));  // (a caller times an empty kernel span)
        if (k_end) HIPCHK(hipEventRecord(k_end, (hipStream_t)stream));
        return GS_OK;
    }
    if (cap >= (int64_t)0xFFFFFFFFll) return fail(GS_ERR_ARG, "partition too large");
    if ((int64_t)cam->image_width * cam->image_height >= (int64_t)0xFFFFFFFFll)
        return fail(GS_ERR_ARG, "image too large for 32-bit pixel ids");
    hipStream_t st = (hipStream_t)stream;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (dev != ds->device) return fail(GS_ERR_ARG, "scene lives on another device");
    KParams kp{};
    kp.sc = ds->dev;
    kp.cam = *cam;
    kp.ss = *ss;
    kp.seed = seed;
    kp.rank = part->rank;
    kp.world_size = part->world_size;
    kp.tile_w = part->tile_w;
    kp.tile_h = part->tile_h;
    kp.tiles_x = (cam->image_width + part->tile_w - 1) / part->tile_w;
    kp.capacity = (uint32_t)cap;
    kp.order = part->d_tile_order;
    // Split pixels into sample chunks only when the settings run exactly one batch:
    // max_samples < batch_size makes the first stop test (camera.rs:158) always true.
    //
    // What the frame's bits depend on (round 6): a pixel's
    // colour is ((0 + C_0) + C_1) + ... over its chunks of c samples, each C_k = ((0 + s) + s)
    // + ... in sample order, so the association is fixed by c alone -- and c is a function of
    // the frame (W x H), the settings, the scene's flags and the process's knobs: never of the
    // rank's capacity, the device count, the device's CUs or a timing.  How the samples are
    // cut into work items is scheduling: the guided tail's 1-sample items (gs_combine_kernel
    // re-forms their chunks of c: a 1-sample chunk sum is 0 + s = s, bit for bit, so the
    // regrouped sum is the coarse chunk's) may sit on any tiles, sized by the rank's capacity,
    // this device's lanes and the scene's measured cost, without changing a bit.
    const int32_t t_sample_chunk = g_sample_chunk.load(std::memory_order_relaxed);
    const uint64_t t_partial_budget = g_partial_budget.load(std::memory_order_relaxed);
    uint32_t chunk = 0, cpp = 1, fine_px = (uint32_t)cap, fine_chunk = 1, fine_cpp = 1;
    if (t_sample_chunk != 0 && ss->max_samples < ss->batch_size) {
        const uint32_t bs = ss->batch_size;
        const uint64_t frame_px = (uint64_t)cam->image_width * (uint64_t)cam->image_height;
        uint32_t c = t_sample_chunk > 0 ? (uint32_t)t_sample_chunk : std::max<uint32_t>(16u, (bs + 63u) / 64u);
        if ((bs + c - 1) / c > 64u) c = (bs + 63u) / 64u;  // at most 64 chunks per pixel
        if (t_sample_chunk < 0)  // (the whole frame's sums: the same c on every rank)
            while (c < bs && frame_px * ((bs + c - 1) / c) * 24u > t_partial_budget) c *= 2u;
        const int32_t t_pct = g_tail_pct.load(std::memory_order_relaxed);
        // A small frame -- at most twice the default tail's samples on a 256-CU device -- of a
        // scene whose samples are alike (no media, no BVHs under instances, no staged shading)
        // runs in chunks of 4 samples: there the items' fixed costs (claims, refills, chunk
        // sums) outweigh the last chunk's length.  MI355X C1 (400x225 x 100 spp, earth + sky):
        // 16-sample chunks with a 2-sample tail on 21 of 28 tiles 14 727, a 4-sample tail 16 579,
        // every tile in 4-sample chunks 18 104 Msamples/s; 3, 5, 6 samples 15 977-17 205
        // (profiles/r05/sweep_C1_guided_tail*.txt).  (A fixed lane count, not this device's:
        // the chunk size is part of what the bits depend on.)
        const bool simple = (ds->feat & (GS_FEAT_MEDIA | GS_FEAT_NESTED | GS_FEAT_MIXED)) == 0;
        const bool small = t_sample_chunk < 0 && t_pct == 0 && simple &&
                           frame_px * bs <= 4ull * (256ull * GS_BLOCK) * std::min(c, bs);
        if (small) c = std::min<uint32_t>(4u, c);
        if (t_sample_chunk < 0 || t_pct > 0) {  // (an explicit chunk with a tail: gs_debug_set_guided_tail)
            // Guided tail: a work item of c samples started just before the queue runs dry
            // can keep its lane busy for c samples while every other lane idles, and a frame
            // with few items per lane ends on them (MI355X final_scene 400x400 x 64 spp,
            // every pixel in chunks of 16: 211 Msamples/s; of 1: 1007).  So the rank's last
            // tiles in queue order run in 1-sample items: enough tiles for 2 x lanes x c
            // samples, which keeps the other lanes busy while the last coarse items finish.
            // A small frame (above) takes no tail while its samples are short: once a frame of
            // the scene measured more than GS_SHORT_SAMPLE_LANE_US lane-microseconds a sample
            // (the frame context, gs_device_scene_note_frame; sticky) it takes the tail too.
            // 400-px reference scenes, tail off / on (profiles/r05/small_frame_rule_scenes.txt),
            // Msamples/s: earth 17 317 / 8 725, hdri 13 956 / 7 100, triangles 14 582 / 8 465,
            // quads 13 402 / 11 088 (17-34 lane-us a sample) -- but checkered_spheres 10 523 /
            // 14 047, cornell_box 8 272 / 8 918, perlin_spheres 1 524 / 3 320, simple_light
            // 1 056 / 2 762 (77-391 lane-us: their last 4-sample items drag the frame).  Being
            // scheduling only, neither the timing nor the device's lanes change a bit.
            c = std::min(c, bs);
            const uint64_t tile_px = (uint64_t)part->tile_w * part->tile_h, slots = (uint64_t)cap / tile_px;
            const uint64_t lanes = (uint64_t)std::max(1, device_cus(dev)) * GS_BLOCK;
            const bool short_samples = !ds->long_samples.load(std::memory_order_relaxed);
            if (c > 1 && slots > 0 && !(small && short_samples)) {
                const uint64_t want = lanes * c * (uint64_t)(t_pct > 0 ? t_pct : 200) / 100u;  // samples
                const uint64_t ft = std::min<uint64_t>(slots, (want + tile_px * bs - 1) / (tile_px * bs));
                const uint32_t fpx = (uint32_t)((slots - ft) * tile_px);
                const uint64_t items = (uint64_t)fpx * ((bs + c - 1) / c) + ((uint64_t)cap - fpx) * bs;
                if (items * 24u <= t_partial_budget && items < 0xFFFFFFFFull) {
                    fine_px = fpx;
                    fine_chunk = 1;
                    fine_cpp = bs;
                }
            }
        }
        if (c < bs || fine_px < (uint32_t)cap) {
            chunk = c;
            cpp = (bs + c - 1) / c;
        }
    }
    if ((uint64_t)fine_px * cpp + ((uint64_t)cap - fine_px) * fine_cpp >= 0xFFFFFFFFull)
        chunk = 0, cpp = 1, fine_px = (uint32_t)cap, fine_cpp = 1;
    if (!chunk) fine_px = (uint32_t)cap, fine_chunk = 1, fine_cpp = 1;
    // Adaptive settings (more than one batch) in batch rounds: rounds = the most batches a
    // pixel can run (the loop ends once sample_count > max_samples, camera.rs:162), in
    // segments of at most seg_px active pixels whose per-sample colours fit the budget.
    uint32_t n_rounds = 0, seg_px = 0, n_segs = 0;
#if defined(GS_STAMPS) || defined(GS_CERT_CHECK)
    const bool visit_out = false;  // (those builds' item_visits is their record buffer: rounds allowed)
#else
    const bool visit_out = outs->item_visits != nullptr;
#endif
    const int32_t t_adaptive = g_adaptive_rounds.load(std::memory_order_relaxed);
    if (t_adaptive && t_sample_chunk != 0 && ss->max_samples >= ss->batch_size && !visit_out && !va) {
        const uint64_t R = (uint64_t)ss->max_samples / ss->batch_size + 1u;
        const uint64_t sp = std::min<uint64_t>((uint64_t)cap, t_partial_budget / ((uint64_t)ss->batch_size * 24u));
        const bool want = t_adaptive == 2 || R * ss->batch_size >= GS_ROUND_MIN_CAP;
        if (want && R <= kMaxRounds && sp >= 1 && sp * ss->batch_size < 0x7FFFFFFFull) {
            n_rounds = (uint32_t)R;
            seg_px = (uint32_t)sp;
            n_segs = (uint32_t)(((uint64_t)cap + sp - 1) / sp);
            chunk = 0;  // (the adaptive lane layout: whole-batch rounds keep Σlum, Σlum², the count)
            cpp = 1;
            fine_px = (uint32_t)cap, fine_chunk = 1, fine_cpp = 1;
        }
    }
    kp.per_sample = n_rounds ? 1u : 0u;
    kp.rounds = n_rounds ? 1u : 0u;
    kp.chunk = chunk;
    kp.cpp = cpp;
    kp.fine_px = fine_px;
    kp.fine_base = fine_px * cpp;
    kp.fine_chunk = fine_chunk;
    kp.fine_cpp = fine_cpp;
    kp.n_items = fine_px * cpp + ((uint32_t)cap - fine_px) * fine_cpp;
    kp.u_cpp = udiv_make(cpp);
    kp.u_fcpp = udiv_make(fine_cpp);
    kp.u_tpx = udiv_make((uint32_t)(part->tile_w * part->tile_h));
    kp.u_bpr = udiv_make(std::max<uint32_t>(1, (uint32_t)part->tile_w >> 3));
    kp.u_tw = udiv_make((uint32_t)part->tile_w);
    kp.u_tx = udiv_make((uint32_t)kp.tiles_x);
    kp.u_w = udiv_make((uint32_t)cam->image_width);
    kp.claim = 1;  // set below, once the grid size is known
    kp.out = outs->rgb;
    kp.out8 = outs->rgb8;
    kp.direct = direct ? 1u : 0u;
    kp.zero_counters = zero_counters && d_counters ? 1u : 0u;
    kp.counters = (unsigned long long*)d_counters;
    kp.item_visits = outs->item_visits;
    kp.visits = va ? va->visits : nullptr;
    kp.visit_leaf_base = va ? va->leaf_base : 0u;
    // (under the scene's mutex from here: the placement pilot's end rewrites the records,
    // the root and the mirror prefixes under it, pilot_end)
    gs_device_scene* mds = const_cast<gs_device_scene*>(ds);
    std::lock_guard<std::mutex> lock(mds->mu);
    KArgs a{};
    a.tnodes = ds->tnodes;
    a.tboxes = ds->tboxes;
    a.tleaves = ds->tleaves;
    a.tquads = ds->tquads;
    a.root = ds->thr_root;
    a.cert_boxes = ds->cert_boxes ? 1 : 0;
    const int32_t t_shade = g_shade_batch.load(std::memory_order_relaxed), t_leaf = g_leaf_batch.load(std::memory_order_relaxed),
                  t_steps = g_node_steps.load(std::memory_order_relaxed);
    a.shade_batch = t_shade > 0 ? t_shade : ds->shade_batch;
    a.leaf_batch = std::max<int32_t>(1, t_leaf > 0 ? t_leaf : ds->leaf_batch);  // (0 would never step a node)
    a.node_steps = std::max(1, std::min<int32_t>(unroll_steps(ds->feat), t_steps > 0 ? t_steps : ds->node_steps));
    const int32_t t_cam = g_cam_batch.load(std::memory_order_relaxed);
    a.cam_batch = std::max<int32_t>(1, t_cam > 0 ? t_cam : ds->cam_batch);
    const bool chunked = kp.chunk != 0;
    gs_device_scene::LaunchCfg& lc = mds->lcfg[chunked ? 1 : 0];
    if (!lc.ready) {
        HIPCHK(hipDeviceGetAttribute(&mds->cus, hipDeviceAttributeMultiprocessorCount, dev));
        // The mirror takes what the block's LDS limit leaves after the kernel's static LDS
        // and the lane state (any prefix of either record array is a valid mirror).
        hipFuncAttributes fa{};
        HIPCHK(hipFuncGetAttributes(&fa, (const void*)kernel_for(ds->feat)));
        int max_lds = 0;
        HIPCHK(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
        // The node mirror must start at LDS address 0 (load_tnode): no static LDS.
        if (fa.sharedSizeBytes != 0) return fail(GS_ERR_UNSUPPORTED, "render kernel with static LDS");
        uint32_t ln = ds->lds_nodes, ll = ds->lds_leaves, lq = ds->lds_quads, lk = ds->lds_cubes;
        auto bytes = [&] {
            return (int64_t)ln * (int64_t)sizeof(TNode) + (int64_t)ll * (int64_t)sizeof(TLeaf) +
                   (int64_t)lq * (int64_t)sizeof(TQuad) + (int64_t)lk * (GS_CUBE_DOUBLES * 8);
        };
        // (the nested walk's save slots too, when they displace no mirror record; else they
        // stay in global memory: final_scene, whose mirror wants more than the 24 KiB the
        // slots would leave, lost 5% with them in LDS -- profiles/r06/ab_nest_save_lds.txt)
        uint32_t nsave = nest_save_lds(ds->feat);
        if ((int64_t)max_lds - (int64_t)lane_lds_bytes(chunked, ds->feat, nsave) < bytes()) nsave = 0;
        const int64_t room = (int64_t)max_lds - (int64_t)lane_lds_bytes(chunked, ds->feat, nsave);
        if (room < 0) return fail(GS_ERR_UNSUPPORTED, "lane state exceeds the device's LDS per block");
        // shrink the least valuable prefix first: cubes, quads, then all
        while (bytes() > room && lk) lk = lk - 1 - lk / 16;
        while (bytes() > room && lq) lq = lq - 1 - lq / 16;
        while (bytes() > room) {
            if (ln) ln = ln - 1 - ln / 16;  // shrink the prefixes until they fit
            if (ll) ll = ll - 1 - ll / 16;
        }
        lc.lds_nodes = ln;
        lc.lds_leaves = ll;
        lc.lds_quads = lq;
        lc.lds_cubes = lk;
        lc.lds = lane_lds_bytes(chunked, ds->feat, nsave) + (size_t)bytes();
        lc.nest_lds = nsave;
        lc.feat = ds->feat;
        if (ln < ds->node_records || ll < ds->leaf_records) lc.feat &= ~GS_FEAT_LDSTREE;
        int occ = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel_for(lc.feat), GS_BLOCK, lc.lds));
        lc.per_cu = occ < 1 ? 1 : (occ > 8 ? 8 : occ);
        lc.ready = true;
    }
    const int cus = ds->cus;
    const size_t lds = lc.lds;
    a.lds_nodes = lc.lds_nodes;
    a.lds_leaves = lc.lds_leaves;
    a.lds_quads = lc.lds_quads;
    a.lds_cubes = lc.lds_cubes;
    a.cubes = ds->dev.cubes;
    a.lane_nd = lane_nd(chunked, ds->feat) + lc.nest_lds;
    a.nest_lds = lc.nest_lds;
    const int32_t t_bpc = g_blocks_per_cu.load(std::memory_order_relaxed);
    const int per_cu = t_bpc > 0 ? t_bpc : lc.per_cu;
    int64_t blocks = (int64_t)cus * per_cu;
    // no more waves than work: one lane per item at most (a round's items: at most one per sample)
    int64_t max_blocks = ((int64_t)(n_rounds ? (uint64_t)seg_px * ss->batch_size : kp.n_items) + GS_BLOCK - 1) / GS_BLOCK;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    // Items per queue claim: about 1/8 of a wave's share of the items, at most 32 (a wave
    // ends holding at most one partly used reserve), at least 1.
    const uint64_t waves = (uint64_t)blocks * (GS_BLOCK / 64);
    kp.waves = (uint32_t)waves;
    kp.lanes = (uint32_t)(blocks * GS_BLOCK);
    // (coarse items of at most 4 samples -- a small frame's chunks -- claim like the tail's: the
    // one queue counter serialises claims of 32; MI355X C1, 4-sample items: 32 -> 1.15 ms, 128 ->
    // 0.57 ms a frame)
    const uint64_t claim_cap = kp.chunk && kp.chunk <= 4u ? (uint64_t)GS_CLAIM_FINE : 32u;
    kp.claim = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(claim_cap, (uint64_t)kp.n_items / waves / GS_CLAIM_DIV));
    kp.claim_fine = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(GS_CLAIM_FINE, (uint64_t)kp.n_items / waves / GS_CLAIM_DIV));
    // The u32 queue counter runs past n_items by at most one claim per wave (each wave's
    // last, failed claim): it must not wrap.
    if ((uint64_t)std::max<uint64_t>(kp.n_items, (uint64_t)seg_px * ss->batch_size) +
            (uint64_t)std::max<uint32_t>(GS_CLAIM_FINE, std::max(kp.claim, kp.claim_fine)) * (waves + 1) >= 0xFFFFFFFFull)
        return fail(GS_ERR_ARG, "too many work items for the 32-bit work queue");

    // This launch's slot.  A slot whose last launch ran on this very stream is reused first:
    // stream order already puts the new launch behind the old one, so one caller on one
    // stream keeps one slot (and one chunk-sum buffer) however many launches it queues.
    // Otherwise a slot whose launch has finished, preferring one whose chunk sums are big
    // enough; otherwise the next in turn, behind a stream wait on its previous launch.
    const size_t need_partial = n_rounds ? (size_t)seg_px * ss->batch_size * 3 * sizeof(double)
                              : chunk ? (size_t)kp.n_items * 3 * sizeof(double) : 0;
    int pick = -1;
    for (int k = 0; k < kLaunchSlots && pick < 0; k++)
        if (mds->slots[k].used && mds->slots[k].stream == st) pick = k;
    if (pick < 0) {
        int idle = -1;
        for (int k = 0; k < kLaunchSlots; k++) {
            LaunchSlot& c = mds->slots[k];
            if (c.used && hipEventQuery(c.done) != hipSuccess) continue;
            if (c.partial_bytes >= need_partial) {
                idle = k;
                break;
            }
            if (idle < 0) idle = k;
        }
        pick = idle >= 0 ? idle : (int)(mds->next_slot++ % kLaunchSlots);
    }
    LaunchSlot& sl = mds->slots[pick];
    if (sl.used && sl.stream != st) HIPCHK(hipStreamWaitEvent(st, sl.done, 0));
    if (chunk || n_rounds) {
        const size_t need = need_partial;
        if (sl.partial_bytes < need) {
            if (sl.used) HIPCHK(hipEventSynchronize(sl.done));  // nothing in flight reads it
            if (sl.partial) (void)hipFree(sl.partial);
            sl.partial = nullptr;
            sl.partial_bytes = 0;
            if (hipMalloc(&sl.partial, need) != hipSuccess)
                return fail(GS_ERR_OOM, "hipMalloc of " + std::to_string(need) + " bytes of chunk sums failed");
            sl.partial_bytes = need;
        }
        kp.partial = sl.partial;
    }
    // batch rounds: [item-size hint, round counts][active list 0][active list 1][running sums],
    // 256-B aligned (the hint first: it outlives launches of other settings)
    const size_t r_counts = ((size_t)(n_rounds + 2) * 4 + 16 + 255) & ~(size_t)255;
    const size_t r_list = ((size_t)cap * 4 + 255) & ~(size_t)255;
    if (n_rounds) {
        const size_t need = r_counts + 2 * r_list + (size_t)cap * 5 * sizeof(double);
        if (sl.rbuf_bytes < need) {
            if (sl.used) HIPCHK(hipEventSynchronize(sl.done));
            if (sl.rbuf) (void)hipFree(sl.rbuf);
            sl.rbuf = nullptr;
            sl.rbuf_bytes = 0;
            if (hipMalloc(&sl.rbuf, need) != hipSuccess)
                return fail(GS_ERR_OOM, "hipMalloc of " + std::to_string(need) + " bytes of batch-round state failed");
            sl.rbuf_bytes = need;
            HIPCHK(hipMemsetAsync(sl.rbuf, 0, 16, st));  // no item-size hint yet
        }
        uint8_t* rb = (uint8_t*)sl.rbuf;
        kp.rpp_hint = (unsigned long long*)rb;
        kp.round_counts = (uint32_t*)(rb + 16);
        kp.active_buf[0] = (uint32_t*)(rb + r_counts);
        kp.active_buf[1] = (uint32_t*)(rb + r_counts + r_list);
        kp.pstate = (double*)(rb + r_counts + 2 * r_list);
    }
    if (lc.feat & GS_FEAT_NESTED) {  // (and the pilot's instantiation, which has every path)
        const size_t need = (size_t)blocks * GS_BLOCK * 64u;
        if (sl.nest_save_bytes < need) {
            if (sl.used) HIPCHK(hipEventSynchronize(sl.done));
            if (sl.nest_save) (void)hipFree(sl.nest_save);
            sl.nest_save = nullptr;
            sl.nest_save_bytes = 0;
            if (hipMalloc(&sl.nest_save, need) != hipSuccess)
                return fail(GS_ERR_OOM, "hipMalloc of " + std::to_string(need) + " bytes of nested-walk save slots failed");
            sl.nest_save_bytes = need;
        }
        kp.nest_save = sl.nest_save;
    }
    kp.queue = sl.queue;
    a.P = sl.params;
    if (outs->item_visits) HIPCHK(hipMemsetAsync(outs->item_visits, 0, (size_t)cap * sizeof(uint32_t), st));
    hipLaunchKernelGGL(gs_params_kernel, dim3(1), dim3(64), 0, st, kp, sl.params);  // (zeroes the queue)
    HIPCHK(hipGetLastError());
#ifndef GS_USE_RSPLIT
#define GS_USE_RSPLIT 1  // (A/B: 0 runs split rounds on the generic instantiation)
#endif
    if (n_rounds) {
        // init (every real packed pixel active), then per round and segment: parameters,
        // the megakernel, the combine; all on the stream, no host synchronisation (a segment
        // or round with no active pixel left launches and exits at once)
        KParams* dP = sl.params;
        HIPCHK(hipMemsetAsync(kp.round_counts, 0, (size_t)(n_rounds + 1) * 4, st));
        const unsigned g_init = (unsigned)std::min<int64_t>((cap + 255) / 256, 8192);
        hipLaunchKernelGGL(gs_round_init_kernel, dim3(g_init), dim3(256), 0, st, (const KParams*)dP);
        HIPCHK(hipGetLastError());
        if (k_begin) HIPCHK(hipEventRecord(k_begin, st));
        const unsigned g_comb = (unsigned)std::min<int64_t>((seg_px + 255) / 256, 8192);
        // Rounds whose items are surely split (gs_round_params_kernel: a requested chunk, a batch
        // above GS_ROUND_WHOLE_MAX_BATCH, or whole-batch items off -- the default) and whose
        // paths always trace a camera ray take the fixed kernel's sample loop (GS_FEAT_RSPLIT).
        const int32_t t_whole = g_round_whole.load(std::memory_order_relaxed);
        const bool rsplit = GS_USE_RSPLIT && has_rsplit(lc.feat) && cam->max_depth > 0 &&
                            (t_sample_chunk > 0 || ss->batch_size > GS_ROUND_WHOLE_MAX_BATCH || t_whole == 0);
        void (*rkern)(KArgs) = kernel_for(rsplit ? lc.feat | GS_FEAT_FIXED | GS_FEAT_RSPLIT : lc.feat);
        for (uint32_t r = 0; r < n_rounds; r++)
            for (uint32_t sg = 0; sg < n_segs; sg++) {
                hipLaunchKernelGGL(gs_round_params_kernel, dim3(1), dim3(64), 0, st, dP, r, sg, seg_px, t_sample_chunk,
                                   t_whole);
                hipLaunchKernelGGL(rkern, dim3((unsigned)blocks), dim3(GS_BLOCK), lds, st, a);
                hipLaunchKernelGGL(gs_round_combine_kernel, dim3(g_comb), dim3(256), 0, st, (const KParams*)dP, r);
            }
        HIPCHK(hipGetLastError());
        if (k_end) HIPCHK(hipEventRecord(k_end, st));
        HIPCHK(hipEventRecord(sl.done, st));
        sl.used = true;
        sl.stream = st;
        return GS_OK;
    }
    if (k_begin) HIPCHK(hipEventRecord(k_begin, st));
    const bool pilot_kernel = va != nullptr;
    // (a fixed-spp chunked launch takes the instantiation without the adaptive paths)
#ifndef GS_USE_FIXED
#define GS_USE_FIXED 1  // (A/B: 0 launches the generic instantiation for fixed-spp frames too)
#endif
    const bool fixed = GS_USE_FIXED && kp.chunk != 0 && !n_rounds && cam->max_depth > 0;
    hipLaunchKernelGGL(kernel_for(pilot_kernel ? GS_FEAT_PILOT : lc.feat | (fixed ? GS_FEAT_FIXED : 0)), dim3((unsigned)blocks),
                       dim3(GS_BLOCK), lds, st, a);
    HIPCHK(hipGetLastError());
    if (k_end) HIPCHK(hipEventRecord(k_end, st));
    if (chunk) {
        const unsigned grid = (unsigned)std::min<int64_t>((cap + 255) / 256, 8192);
        hipLaunchKernelGGL(gs_combine_kernel, dim3(grid), dim3(256), 0, st, (const KParams*)sl.params);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(sl.done, st));
    sl.used = true;
    sl.stream = st;
    return GS_OK;
}

// Placement pilot.  Before a scene's first launch, when its threaded records do not all
// fit the LDS mirror: render the launch's camera at 1 spp on a grid of every k-th pixel
// (k chosen for ~64 k pilot pixels) with the GS_FEAT_VISITS instantiation, which counts
// the tests of every node and leaf record, then re-place the records by measured visits
// per byte (place_records) and upload them again.  The static estimate ranks records by
// geometry alone and misses where the camera's rays actually go (MI355X C4: its mirror
// served 90.8% of node visits and 50.2% of leaf tests; the measured order of the same
// bytes serves 99.6% and 96.0%, tools/visitmap.py).  Placement never changes a result
// (links are explicit), and the pilot is deterministic, so every device of a multi-GPU
// render places its copy identically.
// The pilot in two halves, so a multi-GPU frame issues every device's pilot before it waits
// for any (pilot_begin launches it on the stream, pilot_end waits, reads the counts back and
// re-places the records).
struct PilotRun {
    std::chrono::steady_clock::time_point t0;
    float* d_rgb = nullptr;
    uint32_t* d_vis = nullptr;
    hipStream_t st = nullptr;
    bool launched = false;
};

// The pilot's camera: every k-th pixel of the launch's (~64 k pixels), 1 spp.
static gs_camera pilot_camera(const gs_camera* cam) {
    const int64_t px = (int64_t)cam->image_width * cam->image_height;
    const int32_t k = std::max<int32_t>(1, (int32_t)std::sqrt((double)px / 65536.0));
    gs_camera pc = *cam;
    pc.image_width = (cam->image_width + k - 1) / k;
    pc.image_height = (cam->image_height + k - 1) / k;
    for (int a = 0; a < 3; a++) {
        pc.pixel_delta_u[a] = cam->pixel_delta_u[a] * (double)k;
        pc.pixel_delta_v[a] = cam->pixel_delta_v[a] * (double)k;
    }
    return pc;
}

static gs_status pilot_begin(gs_device_scene* ds, const gs_camera* cam, void* stream, PilotRun& pr) {
    pr.t0 = std::chrono::steady_clock::now();
    const gs_camera pc = pilot_camera(cam);
    gs_partition part{0, 1, 64, 64, nullptr, 0, 0};
    const int64_t cap = gs_partition_capacity(&pc, &part);
    const uint32_t nn = ds->node_records, nl = ds->leaf_records;
    if (hipMalloc(&pr.d_rgb, (size_t)cap * 12 + 16) != hipSuccess ||
        hipMalloc(&pr.d_vis, ((size_t)nn + nl) * 4 + 16) != hipSuccess) {
        if (pr.d_rgb) (void)hipFree(pr.d_rgb);
        pr.d_rgb = nullptr;
        return fail(GS_ERR_OOM, "hipMalloc of the placement pilot's buffers failed");
    }
    pr.st = (hipStream_t)stream;
    gs_sample_settings one{0.0, 0.0, 1, 0};  // one sample per pixel (camera.rs:158: max_samples < batch)
    gs_render_outputs o{pr.d_rgb, nullptr, nullptr};
    VisitArgs va{pr.d_vis, nn};
    hipError_t e = hipMemsetAsync(pr.d_vis, 0, ((size_t)nn + nl) * 4, pr.st);
    gs_status r = e == hipSuccess ? launch(ds, &pc, &one, 1, &part, &o, nullptr, stream, nullptr, nullptr, &va)
                                  : fail(GS_ERR_HIP, hipGetErrorString(e));
    pr.launched = r == GS_OK;
    return r;
}

static gs_status pilot_end(gs_device_scene* ds, PilotRun& pr) {
    const uint32_t nn = ds->node_records, nl = ds->leaf_records;
    std::vector<uint32_t> vis((size_t)nn + nl);
    gs_status r = GS_OK;
    if (pr.launched) {
        hipError_t e = hipStreamSynchronize(pr.st);
        if (e == hipSuccess) e = hipMemcpy(vis.data(), pr.d_vis, vis.size() * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) r = fail(GS_ERR_HIP, std::string("placement pilot: ") + hipGetErrorString(e));
    }
    if (pr.d_rgb) (void)hipFree(pr.d_rgb);
    if (pr.d_vis) (void)hipFree(pr.d_vis);
    pr.d_rgb = nullptr;
    pr.d_vis = nullptr;
    if (!pr.launched) return fail(GS_ERR_HIP, "placement pilot not launched");
    if (r != GS_OK) return r;
    const ThreadedTree& t = ds->tree;
    std::vector<uint64_t> counts(t.rec.size());
    for (size_t i = 0; i < t.rec.size(); i++) counts[i] = t.leaf[i] ? vis[(size_t)nn + ds->pos[i]] : vis[ds->pos[i]];
    Placed pl = place_records(t, &counts, ds->single_quads, ds->mirror_budget, ds->nroot_rec, ds->n_cubes);
    if (pl.tnodes.size() != nn || pl.tleaves.size() != nl) return fail(GS_ERR_HIP, "placement changed the record counts");
    {
        // The arrays are rewritten in place, so nothing of this scene may be running: the
        // pilot is not always the scene's first launch (pilot_due defers it past small ones,
        // which may still be in flight on other streams).  Every launch records its slot's
        // `done` event under `mu` before it returns, so with `mu` held every launch enqueued
        // so far has an event to wait for, and none can start until the records and the
        // launch shape below agree again.
        std::lock_guard<std::mutex> lock(ds->mu);
        for (int k = 0; k < kLaunchSlots; k++)
            if (ds->slots[k].used) HIPCHK(hipEventSynchronize(ds->slots[k].done));
        HIPCHK(hipMemcpy(const_cast<TNode*>(ds->tnodes), pl.tnodes.data(), pl.tnodes.size() * sizeof(TNode),
                         hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(const_cast<TBox*>(ds->tboxes), pl.tboxes.data(), pl.tboxes.size() * sizeof(TBox),
                         hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(const_cast<TLeaf*>(ds->tleaves), pl.tleaves.data(), pl.tleaves.size() * sizeof(TLeaf),
                         hipMemcpyHostToDevice));
        if (!pl.nroots.empty())
            HIPCHK(hipMemcpy(ds->nroots, pl.nroots.data(), pl.nroots.size() * 4, hipMemcpyHostToDevice));
        ds->thr_root = pl.root;
        ds->lds_nodes = pl.lds_nodes;
        ds->lds_leaves = pl.lds_leaves;
        ds->lds_quads = pl.lds_quads;
        ds->lds_cubes = pl.lds_cubes;
        ds->pos = std::move(pl.pos);
        ds->lcfg[0].ready = ds->lcfg[1].ready = false;  // mirror prefixes changed
    }
    ds->pilot_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - pr.t0).count();
    ds->tree = ThreadedTree{};  // not needed again
    ds->placement.store(2, std::memory_order_release);
    return GS_OK;
}

// Does this launch run the scene's pending pilot?  Not when placement is settled, or every
// record is mirrored anyway (then it is settled as static), and not yet when the launch is
// small next to the pilot: a pilot of ~64 k pixel samples before a launch of fewer than
// 16 x as many samples costs more than a better mirror can save there (a one-shot 4-spp
// frame of <= 64 k pixels would pay a full-frame pass, +25%), so it waits for a bigger one.
static bool pilot_due(gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss) {
    if (ds->placement.load(std::memory_order_acquire) != 0) return false;
    const bool all_mirrored = ds->lds_nodes == ds->node_records && ds->lds_leaves == ds->leaf_records;
    // (scenes of the catch-all kernel keep the static placement: the pilot's instantiation does
    // not walk their compositions)
    if (!g_placement || all_mirrored || !cam || cam->image_width <= 0 || cam->image_height <= 0 ||
        (ds->feat & GS_FEAT_GENERAL)) {
        ds->placement.store(1, std::memory_order_release);
        return false;
    }
    const gs_camera pc = pilot_camera(cam);
    const uint64_t pilot_samples = (uint64_t)pc.image_width * (uint64_t)pc.image_height;
    const uint64_t samples = (uint64_t)cam->image_width * (uint64_t)cam->image_height * (ss ? ss->batch_size : 1u);
    return samples >= 16u * pilot_samples;
}

static gs_status ensure_placement(gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                  void* stream) {
    if (ds->placement.load(std::memory_order_acquire) != 0) return GS_OK;
    std::lock_guard<std::mutex> g(ds->place_mu);
    if (!pilot_due(ds, cam, ss)) return GS_OK;
    PilotRun pr;
    gs_status r = pilot_begin(ds, cam, stream, pr);
    const gs_status r2 = pilot_end(ds, pr);  // (frees the buffers either way; tried again at the next launch)
    return r != GS_OK ? r : r2;
}

// The frame context's first frame (and camera changes): every device's pending pilot is
// launched before any is waited for, so N devices pilot concurrently (internal.hpp).
gs_status gs_placement_prepare(gs_device_scene* const* scenes, const int* devices, void* const* streams, int n,
                               const gs_camera* cam, const gs_sample_settings* ss, int* ran) {
    *ran = 0;
    std::vector<std::unique_lock<std::mutex>> locks;
    std::vector<PilotRun> runs(n);
    std::vector<int> due(n, 0);
    gs_status r = GS_OK;
    for (int i = 0; i < n && r == GS_OK; i++) {
        gs_device_scene* ds = scenes[i];
        if (ds->placement.load(std::memory_order_acquire) != 0) continue;
        locks.emplace_back(ds->place_mu);
        if (!pilot_due(ds, cam, ss)) continue;
        if (hipSetDevice(devices[i]) != hipSuccess) {
            r = fail(GS_ERR_HIP, "hipSetDevice failed");
            break;
        }
        due[i] = 1;
        *ran = 1;
        r = pilot_begin(ds, cam, streams[i], runs[i]);
    }
    for (int i = 0; i < n; i++) {
        if (!due[i]) continue;
        (void)hipSetDevice(devices[i]);
        const gs_status e = pilot_end(scenes[i], runs[i]);
        if (r == GS_OK) r = e;
    }
    return r;
}

extern "C" {

gs_status gs_plan_tiles(const gs_device_scene* ds, const gs_camera* cam, uint64_t seed, int32_t world,
                        int32_t tile_w, int32_t tile_h, int32_t* order_out, int64_t order_cap,
                        int32_t* slots_per_rank) {
    if (!ds || !cam || !slots_per_rank || world < 1 || tile_w < 1 || tile_h < 1)
        return fail(GS_ERR_ARG, "bad argument");
    gs_partition all{0, 1, tile_w, tile_h, nullptr, 0, 0};
    if (!part_ok(cam, &all)) return fail(GS_ERR_ARG, "bad partition / image size");
    const int32_t tx = (cam->image_width + tile_w - 1) / tile_w, ty = (cam->image_height + tile_h - 1) / tile_h;
    const int32_t nt = tx * ty;
    const int32_t slots = (nt + world - 1) / world;  // LPT below never gives a rank more (see the cap)
    if (!order_out) {
        *slots_per_rank = slots;
        return GS_OK;
    }
    // 1-spp pilot over the whole frame: per-pixel BVH node visits (deterministic).
    const int64_t cap = gs_partition_capacity(cam, &all);
    float* d_rgb = nullptr;
    uint32_t* d_vis = nullptr;
    if (hipMalloc(&d_rgb, (size_t)cap * 12 + 16) != hipSuccess || hipMalloc(&d_vis, (size_t)cap * 4 + 16) != hipSuccess) {
        if (d_rgb) (void)hipFree(d_rgb);
        return fail(GS_ERR_OOM, "hipMalloc failed");
    }
    gs_sample_settings one{0.0, 0.0, 1, 0};
    gs_render_outputs o{d_rgb, nullptr, d_vis};
    gs_status r = gs_render_tiles_ex_async(ds, cam, &one, seed, &all, &o, nullptr, nullptr);
    std::vector<uint32_t> vis((size_t)cap);
    if (r == GS_OK) {
        hipError_t e = hipStreamSynchronize(nullptr);  // (the launch's stream: this device's alone)
        if (e == hipSuccess) e = hipMemcpy(vis.data(), d_vis, (size_t)cap * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) r = fail(GS_ERR_HIP, hipGetErrorString(e));
    }
    (void)hipFree(d_rgb);
    (void)hipFree(d_vis);
    if (r != GS_OK) return r;
    // Tile cost: node visits + a per-path constant (shading, camera ray), over real pixels.
    const int64_t tpx = (int64_t)tile_w * tile_h;
    std::vector<double> cost(nt, 0.0);
    for (int32_t t = 0; t < nt; t++) {
        const int32_t x0 = (t % tx) * tile_w, y0 = (t / tx) * tile_h;
        for (int32_t y = 0; y < tile_h; y++)
            for (int32_t x = 0; x < tile_w; x++)
                if (x0 + x < cam->image_width && y0 + y < cam->image_height)
                    cost[t] += 16.0 + (double)vis[(size_t)t * tpx + (size_t)y * tile_w + x];
    }
    // Longest processing time first: the costliest tile to the least-loaded rank (ties:
    // lowest rank) among ranks with a free slot.
    std::vector<int32_t> idx(nt);
    for (int32_t t = 0; t < nt; t++) idx[t] = t;
    std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return cost[a] > cost[b]; });
    std::vector<double> load(world, 0.0);
    std::vector<std::vector<int32_t>> lists(world);
    for (int32_t t : idx) {
        int32_t best = -1;
        for (int32_t rk = 0; rk < world; rk++)
            if ((int32_t)lists[rk].size() < slots && (best < 0 || load[rk] < load[best])) best = rk;
        lists[best].push_back(t);
        load[best] += cost[t];
    }
    // Each rank walks its tiles in frame order: measured on MI355X (C4, 8 ranks) frame
    // order beat descending cost (max rank 87.6 vs 88.0 ms, mean 85.0 vs 86.5): locality
    // between neighbouring tiles outweighs ending the queue on cheap tiles.
    for (auto& l : lists) std::sort(l.begin(), l.end());
    if (order_cap < (int64_t)slots * world) return fail(GS_ERR_ARG, "order_out too small");
    for (int32_t sl = 0; sl < slots; sl++)
        for (int32_t rk = 0; rk < world; rk++)
            order_out[(size_t)sl * world + rk] = sl < (int32_t)lists[rk].size() ? lists[rk][sl] : -1;
    *slots_per_rank = slots;
    return GS_OK;
}

gs_status gs_debug_record_visits(const gs_device_scene* ds, const gs_camera* cam, const gs_sample_settings* ss,
                                 uint64_t seed, const gs_partition* part, float* d_packed_rgb, uint32_t* d_visits,
                                 void* stream) {
    if (!ds || !cam || !d_packed_rgb || !d_visits) return fail(GS_ERR_ARG, "null argument");
    gs_status e = ensure_placement(const_cast<gs_device_scene*>(ds), cam, ss, stream);
    if (e != GS_OK) return e;
    HIPCHK(hipMemsetAsync(d_visits, 0, ((size_t)ds->node_records + ds->leaf_records) * 4, (hipStream_t)stream));
    gs_render_outputs o{d_packed_rgb, nullptr, nullptr};
    VisitArgs va{d_visits, ds->node_records};
    return launch(ds, cam, ss, seed, part, &o, nullptr, stream, nullptr, nullptr, &va);
}

gs_status gs_device_alloc(int64_t bytes, void** d_out) {
    if (!d_out || bytes < 0) return fail(GS_ERR_ARG, "bad argument");
    *d_out = nullptr;
    if (hipMalloc(d_out, (size_t)std::max<int64_t>(bytes, 1)) != hipSuccess) return fail(GS_ERR_OOM, "hipMalloc failed");
    return GS_OK;
}
gs_status gs_device_free(void* d) {
    if (d) HIPCHK(hipFree(d));
    return GS_OK;
}
gs_status gs_device_upload(void* d_dst, const void* src, int64_t bytes) {
    if (!d_dst || !src || bytes < 0) return fail(GS_ERR_ARG, "bad argument");
    HIPCHK(hipMemcpy(d_dst, src, (size_t)bytes, hipMemcpyHostToDevice));
    return GS_OK;
}
gs_status gs_device_download(void* dst, const void* d_src, int64_t bytes) {
    if (!dst || !d_src || bytes < 0) return fail(GS_ERR_ARG, "bad argument");
    HIPCHK(hipMemcpy(dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost));
    return GS_OK;
}

}  // extern "C"
