// iqpt_internal.hpp — types shared by the runtime (iqpt_runtime.cpp) and the kernels
// (iqpt_kernels.hip), plus the error plumbing of the C ABI.
#pragma once

#include <cstdint>
#include <string>

#include "iqpt.h"

namespace iqpt {

// Thread-local detail string behind iqpt_last_error() (the C-ABI counterpart of
// renderer_base::cuda_exception::what, renderer_base.cu:118-128).
void set_last_error(const std::string& msg);
int fail(int status, const std::string& msg);

// 16-byte vector storage usable from plain host C++ (the kernels view it as float4).
struct alignas(16) float4_storage {
    float x, y, z, w;
};

// Device layout of the scene (world space, built once per packet upload):
//  * single triangles, 3 x float4 = 48 B:
//      (v0.x, v0.y, v0.z, e1.x), (e1.y, e1.z, e2.x, e2.y), (e2.z, 0, 0, 0)
//    with v0 the world-space first vertex and e1 = v1 - v0, e2 = v2 - v0 (shape.cu:65-66);
//  * triangle PAIRS (2k, 2k+1), SoA inside the pair, 5 x float4 = 80 B, so that one packed
//    (v_pk_*_f32) instruction advances both Möller–Trumbore tests and every operand pair lands in
//    an aligned VGPR pair straight from one ds_read_b128:
//      (v0x_a, v0x_b, v0y_a, v0y_b), (v0z_a, v0z_b, e1x_a, e1x_b), (e1y_a, e1y_b, e1z_a, e1z_b),
//      (e2x_a, e2x_b, e2y_a, e2y_b), (e2z_a, e2z_b, 0, 0)
//    an odd last triangle is paired with a zero triangle that is masked out;
//  * spheres: (center.xyz, radius) float4, and sphere pairs 2 x float4 = 32 B:
//      (cx_a, cx_b, cy_a, cy_b), (cz_a, cz_b, r_a, r_b).
constexpr int kTriFloat4 = 3;
constexpr int kBvhNodeFloat4 = 4;     // 64 bytes: one cache line per node visit
constexpr int kTriPairFloat4 = 5;
constexpr int kSphPairFloat4 = 2;
// Shading record per triangle (only read for the closest hit): world normals n0, n1, n2 and the
// geometric normal e1 x e2 (shape.cu:96-101) packed in the w lanes — 3 x float4. Not read under
// the reference's hard-wired materials (every triangle is emissive, path_tracer.cu:278), kept for
// the per-primitive material table.
constexpr int kTriShadeFloat4 = 3;

// Kernel parameters (passed by value; lands in SGPRs / the kernarg segment).
struct kparams {
    uint32_t width, height;          // full frame (camera + global pixel id)
    uint32_t x0, ncols;              // owned columns [x0, x0 + ncols)
    uint32_t y0, ystep, nrows;       // owned rows y0 + k * ystep
    uint32_t npix;                   // ncols * nrows
    uint64_t frame0;                 // frames accumulated before this launch
    uint32_t spp;                    // samples per pixel in this launch
    int32_t max_depth;
    float inv_proj[16];              // camera.h:30-31 (row-major m[r][c])
    float inv_view[16];
    uint32_t cam_const;              // inverse projection has constant w (see camera_ray)
    float cam_near_rw, cam_far_rw;   // 1 / w_near, 1 / w_far when cam_const
    float rcp_width, rcp_height;     // RN(1 / W), RN(1 / H) (kOptFastDiv camera divisions)
    // kOptCamAxis (camera_ray_axis): P[0], P[5], P[12], P[13], 1/w_near, 1/w_far, V[0], V[12], V[5],
    // V[6], V[13], V[14], then the launch constants z_n V[9], z_f V[9], z_n V[10], z_f V[10]
    // (z_n, z_f: unprojected z of the near / far point divided by its w)
    float cam_ax[16];
    uint32_t acc_tab;                // build the per-launch (1/n, (n-1)/n) table in LDS
    uint32_t frames32;               // frame0 + spp < 2^32: 32-bit frame-counter conversions
    float mean_tiny;                 // kOptFastDiv running mean: c below this takes the IEEE division
    const float4_storage* tris;      // ntri * kTriFloat4 (single layout)
    const float4_storage* tri_pairs; // ntri_pairs * kTriPairFloat4 (pair layout)
    uint32_t ntri, ntri_pairs;
    const float4_storage* spheres;   // nsph (center.xyz, radius)
    const float4_storage* sph_pairs; // nsph_pairs * kSphPairFloat4
    uint32_t nsph, nsph_pairs;
    uint32_t tri_batch;              // LDS batch (triangles or triangle pairs, by layout)
    uint32_t sph_batch;              // LDS batch (spheres or sphere pairs, by layout)
    float4_storage* lin;             // npix
    uint32_t* bgra;                  // npix, compact row-major order (tile_to_compact), possibly padded after npix
    uint32_t* rng;                   // 6 planes of npix words: v0..v4, d
    unsigned long long* rays;        // closest-hit query counters: kRaySlots slots, kRaySlotStride apart (summed on read)
    uint32_t* queue;                 // tile dequeue head (zeroed before every launch)
    unsigned long long* stats;       // kOptStats counters (8 x u64) or null
    // kOptCull: per screen tile of kCullTile x kCullTile owned pixels (columns x owned rows), one bit
    // per triangle pair (words [0, cull_wt)) and per sphere pair (words [cull_wt, cull_stride)) that
    // camera rays of the tile may hit (iq_interval.h); null = no culling for this launch
    const uint32_t* cull;
    uint32_t cull_ntx, cull_wt, cull_stride;
    // per tile, two words: the 64-bit mask of its pixels (storage order inside the tile) whose every camera
    // ray is certain to end on an emissive triangle (no sphere candidate in the tile, a candidate triangle
    // every ray of the pixel's bundle hits: iq_interval.h tri_certain; the reference's materials only);
    // null = none. Such a pixel's samples are (1, 1, 1) folds and two draws each.
    const uint32_t* certain;
    // per tile, two words: the 64-bit mask of its pixels whose every camera ray is certain to miss every
    // primitive (the pixel's own bundle culls each candidate, iq_interval.h): their samples are the sky
    // gradient of the camera ray, rendered by iqpt_sky_kernel; the plain kernel skips them. null = none.
    const uint32_t* miss;
    // work queue over tiles: queue position q -> tile tile_order[q] (null = identity); built with the
    // masks, most expensive tiles first (longest-processing-time order: a shorter launch tail)
    const uint32_t* tile_order;
    uint32_t ntx, ntiles;            // tiles of the owned set (kCullTile x kCullTile)
    // candidate lists of the masks (streamed scenes): ascending pair indices of tile t's set bits at
    // list[off_tri[t] .. off_tri[t + 1]) and list[off_sph[t] .. off_sph[t + 1]); null = none
    const uint32_t* list;
    const uint32_t* list_off_tri;
    const uint32_t* list_off_sph;
    // per-pixel candidate masks over the tile's triangle list (round 6, iqpt_pixel_mask_kernel): bit e of word w of
    // pixel i (tile storage order) of tile t, at pmask[pmask_off[t] + 64 w + i], is set unless the pixel's own bundle
    // culls both triangles of list entry 32 w + e; tiles whose list is longer than kPixMaskMax entries have none (the
    // wave-uniform list loop). null = none
    const uint32_t* pmask;
    const uint32_t* pmask_off;
    // per tile (2 words): the pixels one of whose tile's candidate triangles accepts every camera ray of the pixel
    // (iq_interval.h tri_certain), for iqpt_anyhit_kernel (any-hit scenes: such a pixel ends every sample on its
    // camera ray with the emissive colour)
    const uint32_t* pmask_certain;
    // kOptMaterials (packet material table): material index per triangle / sphere, the material
    // records (2 x float4 each: (albedo.rgb, type bits), (strength | sigma, A, B, 0)) and the
    // triangle shading records (kTriShadeFloat4 per triangle)
    const uint32_t* tri_mat;
    const uint32_t* sph_mat;
    const float4_storage* mats;
    const float4_storage* tri_shade;
    // exact BVH for secondary rays (iq_bvh.hpp; streamed scenes): nodes (kBvhNodeFloat4 x float4:
    // (tight box min, link: skip pointer or 1 << 31 | leaf first pair << 8 | count), (box max, tA | tB
    // bf16 rounded up), (normal-cone axis, E_det), (gR, gB, Nmin cos beta, Nmin sin beta)), leaf triangle
    // pairs (kTriPairFloat4 each; the packet indices in the last float4's z, w, ~0u pads), triangles outside the
    // BVH (tested by every ray); the bound holds for |d_i| <= md and a finite origin; gulp covers the
    // rounding of a grown box side
    const float4_storage* bvh_nodes;
    const float4_storage* bvh_pairs;
    const uint32_t* bvh_always;
    uint32_t bvh_nnodes, bvh_nalways;
    float bvh_md, bvh_gulp;
    // exact sphere BVH (iq_bvh.hpp, streamed scenes with many spheres): nodes (kSphNodeFloat4 x float4:
    // box min + skip, box max + leaf first << 8 | count, (r_min, r_max, -, -)), leaf spheres (centre,
    // radius) with their packet indices, spheres outside the BVH (tested by every ray)
    const float4_storage* sbvh_nodes;
    const float4_storage* sbvh_sph;
    const uint32_t* sbvh_idx;
    const uint32_t* sbvh_always;
    uint32_t sbvh_nnodes, sbvh_nalways;
    float sbvh_gulp;
    // kOptSplit: sample-parallel chains. A "split pixel" sp (slot sp of the split set,
    // split tile sp / 64, pixel sp % 64 of that tile) whose chains are long ("heavy": its last launch
    // took >= heavy_rho slots per sample) has a sample evaluated speculatively at every even RNG offset
    // 2j ("slot" j) of a window of M slots in round 1, by runs of R consecutive slots, and the chain is
    // stitched in order by iqpt_split_stitch_kernel; the split tiles' light pixels run anchored; a chain
    // that leaves its window is finished by an anchored lane in round 2.
    uint32_t split_round;            // 1: runs + anchored tiles + light split pixels, 2: anchored leftovers
    uint32_t n_anchor;               // round 1: the anchored tiles anchor_order[]
    const uint32_t* anchor_order;
    uint32_t n_split_tiles;
    const uint32_t* split_tiles;     // split tile -> tile index
    const uint32_t* chunks;          // round 1 run chunks (tile, split tile | run << 23), built by the prep
    const uint32_t* chunk_count;
    uint32_t split_len;              // R: slots per run
    uint32_t refill_min;             // idle lanes before a refill (1 = every iteration with an idle lane)
    uint32_t ns_cap, m_cap;          // split pixel slots (split tiles x 64); window cap (multiple of 16)
    const uint32_t* sp_win;          // M of a heavy pixel's window this launch, 0 for a light pixel
    uint32_t* sp_rho;                // slots per sample of the pixel's last chain, x 256 (0 = none)
    const uint32_t* run_st;          // (G_max + 1) x 6 planes of ns_cap words: state at slot r R, at M (plane G_max)
    float4_storage* res;             // res[sp * m_cap + j]: clamped colour, slots consumed (uint bits in w)
    uint8_t* nres;                   // nres[sp * m_cap + j]: slots consumed (the stitch's walk)
    const uint32_t* left;            // round 2: leftover split slots
    const uint32_t* left_count;
    const uint32_t* sp_pix;          // storage index of split slot sp (~0u: no pixel)
    const uint32_t* sp_st;           // 6 planes of ns_cap: a leftover's state at its chain position
    const float4_storage* sp_acc;    // a leftover's accumulator, samples done (uint bits in w)
    // kOptOverlap: consecutive launches run concurrently on two streams. Every tile is
    // bound to one XCD (its L2 is the coherence point of the tile's pixel state): an XCD's waves take
    // only its own tiles, xcd_order[xcd_off[x] + q] in cost order, from the queue word queue[16 x].
    // Launch k of an overlap chain takes tile t once tile_done[t] >= k * pixels(t) (every earlier
    // launch of the chain finished the tile) and adds its completed pixels after their stores.
    uint32_t* tile_done;
    uint32_t done_target;            // k: launches of the chain before this one (0: no wait)
    const uint32_t* xcd_order;
    uint32_t xcd_off[9];
    uint32_t* ovl_err;               // bit 0: a wait exceeded spin_limit, bit 2: an XCD's tile list was never taken
                                     // (no workgroup ran there)
    // forward-progress bound (never reached by a real launch; iqpt_debug_set_limits lowers it so that tests can
    // force it): s_sleep polls of one per-tile wait; iter_limit bounded the archived chain kernel's loop (unused)
    uint32_t spin_limit, iter_limit;
    // iqpt_fan_kernel: the lanes of fan tile b that it renders (bit i: pixel i of the tile); null = all.
    // Spec launches give the fan kernel every pixel whose camera rays provably miss every sphere, also
    // inside tiles with sphere candidates (the other pixels of those tiles are the spec kernel's).
    const uint64_t* fan_lanes;
    // queue length of the plain kernel's tile queue (tile_order[0 .. nqueue)); 0: every tile (ntiles).
    // Chain launches give the plain kernel the anchored tiles only.
    uint32_t nqueue;
    // any-hit scene: no sphere and the reference's hard-wired materials, so every triangle is emissive
    // (path_tracer.cu:278) and every accepted triangle ends the path with the same clamped colour: a ray's
    // result depends only on whether some triangle accepts it, not on which one is closest. The BVH traversal
    // and the candidate-list loop then stop at the first accepted triangle (C4).
    uint32_t anyhit;
};
// The ray count is spread over kRaySlots counters 128 B apart: thousands of waves add their counts as
// they end, and one counter would serialise those atomics at the end of every launch.
constexpr uint32_t kRaySlots = 64;
constexpr uint32_t kRaySlotStride = 16;      // unsigned long longs
constexpr int kSphNodeFloat4 = 3;
constexpr uint32_t kOverlapSpinLimit = 1u << 23;   // s_sleep(20) polls before a wait gives up (~seconds)
constexpr uint32_t kChainIterLimit = 1u << 22;     // (the archived chain kernel's loop bound; iqpt_debug_set_limits)
// two launch parities x (8 XCD queue words + the finished-block count), 64 B apart
constexpr uint32_t kOverlapQueueWords = 2 * 9 * 16;

// Slot-parallel sphere pixels (IQPT_SPLIT_SPEC): the pixels whose own camera-ray bundle
// may reach a sphere. Per launch a window of M slots per pixel (M from the pixel's last chain), every
// slot j (the sample that starts 2j draws into the pixel's stream) evaluated in parallel, 16 lanes per
// pixel, then the chain walked in order (iqpt_spec_kernel).
struct kspec {
    uint32_t n;                      // sphere pixels q < n
    uint32_t m_cap;                  // window cap (a multiple of 16)
    uint32_t rho0;                   // slots per sample x 256 assumed for a pixel without history
    uint32_t margin_div;             // spec_window's margin: 1 / margin_div of the extra slots
    const uint32_t* pix;             // tile-major storage index of sphere pixel q
    uint32_t* m;                     // the last launch's window of q (statistics)
    uint32_t* rho;                   // slots per sample x 256 of q's last chain (0: none)
    uint32_t* run_count;             // [1]: chains finished past their window (statistics)
    float4_storage* res;             // res[q m_cap + j]: clamped colour of slot j
    // parity pixels: round 0 of a pixel whose last chain took >= parity_rho / 256 slots
    // per sample traces the even slots of its window first, the odd ones only from where its chain lands on
    // one (pooled over the block's lanes); 0: every slot of every window
    uint32_t parity_rho;
    uint32_t parity_hi;              // ... and at most parity_hi / 256 slots per sample
    const uint32_t* order;           // a plan (else null): sphere pixel q at each position, heaviest first
    const uint32_t* blocks;          // per plan block: first position, count | log2(lanes / 8) << 8
    uint32_t nblocks;                // plan blocks (the spec part of the grid)
    unsigned long long* tl;          // measurement (iqpt_debug_spec_timeline), else null: per spec block
                                     // s_memrealtime at start, after round 0's slots and walk, at the end
                                     // (| rounds << 48)
};
constexpr int kSendRing = 4;                // the multi-GPU gather's send buffers, used in turn
constexpr int kPipeRing = 6;                // frame buffers pipelined launches write in turn once copies follow them
constexpr int kGatherCtas = 2;              // RCCL blocks per frame gather (iqpt_debug_set_gather)
constexpr uint32_t kSpecReplan = 64;        // launches between two spec plans (the history read behind them)
constexpr uint32_t kSpecPixPerBlock = 16;   // sphere pixels per iqpt_spec_kernel block without a plan (16 lanes each)
constexpr uint32_t kSpecMaxPixPerBlock = 32;   // a plan's blocks: 256 / (8, 16, 24, 32, 48 or 64) pixels
constexpr uint32_t kSpecBlockLanes = 256;      // iqpt_spec_kernel's block
constexpr int kSpecLaneClasses = 4;            // lanes per pixel: 8, 16, 32, 64 (round 4's 24 and 48 split waves)
constexpr uint32_t kSpecRho0 = 576;      // 2.25 slots per sample before a pixel has a history (sphere pixels take ~2)
constexpr uint32_t kSpecParityRho = 480; // parity pixels: >= 1.875 slots per sample in their last chain (kspec::parity_rho)
constexpr uint32_t kSpecParityHi = 528;  // ... and <= 2.0625 (kspec::parity_hi)

// The spec window of a sphere pixel whose last chain used rho256 / 256 slots per sample: that many slots
// for spp samples plus a margin of 1 / margin_div of the extra slots (at least 4) and 4, within
// [spp, m_cap]. A chain longer than its window is finished sequentially by the stitch.
__host__ __device__ inline uint32_t spec_window(uint32_t rho256, uint32_t spp, uint32_t m_cap, uint32_t margin_div) {
    const uint64_t m = ((uint64_t)spp * rho256 + 255u) / 256u;
    const uint64_t extra = m > spp ? (m - spp) / (margin_div ? margin_div : 1u) : 0u;
    uint64_t w = m + (extra > 4u ? extra : 4u) + 4u;
    if (w < spp) w = spp;
    return (uint32_t)(w > m_cap ? m_cap : w);
}

// iqpt_split_prep_kernel / iqpt_split_stitch_kernel (kOptSplit).
struct ksplit {
    uint32_t ns_cap, spp, m_cap, g_max, run_len, heavy_rho;
    uint32_t ncols, nrows;           // the owned set (the BGRA8 frame's compact order)
    int32_t max_depth;
    uint64_t frame0;
    float mean_tiny;
    uint32_t npix;
    const uint32_t* sp_pix;
    uint32_t* sp_win;
    uint32_t* sp_rho;                // slots per sample of the pixel's last completed chain, x 256 (0 = none)
    uint32_t* run_st;
    const uint32_t* split_tiles;
    uint32_t* chunks;
    uint32_t* chunk_count;
    const float4_storage* res;
    const uint8_t* nres;
    uint32_t* left;
    uint32_t* left_count;
    uint32_t* sp_st;
    float4_storage* sp_acc;
    float4_storage* lin;
    uint32_t* bgra;
    uint32_t* rng;
    unsigned long long* rays;
};
constexpr uint32_t kSplitMCapMul = 3;    // window cap M <= 3 spp (rounded up to 16)
constexpr uint32_t kSplitRunLen = 8;     // R: slots per speculative run
constexpr uint32_t kSplitHeavyRho = 320; // heavy pixel: >= 1.25 slots per sample last launch (x 256)

// The window of a split pixel for a launch of spp samples: its last chain's slots per sample rho
// (x 256) times spp, plus a margin of an eighth of the extra slots (at least 2), + 2; 1.5 spp without
// history; within [spp, m_cap]. Round 1 and the stitch both use this value (through sp_win).
__host__ __device__ inline uint32_t split_window(uint32_t rho256, uint32_t spp, uint32_t m_cap) {
    if (rho256 == 0u) return spp + spp / 2u > m_cap ? m_cap : spp + spp / 2u;
    const uint64_t m = ((uint64_t)spp * rho256 + 255u) / 256u;
    const uint64_t extra = m > spp ? (m - spp) / 8u : 0u;
    uint64_t w = m + (extra > 2u ? extra : 2u) + 2u;
    if (w < spp) w = spp;
    return (uint32_t)(w > m_cap ? m_cap : w);
}

// Binning launch (iqpt_bin_kernel): the camera and pixel set of the context, the world-space scene.
struct kbin {
    uint32_t width, height, x0, ncols, y0, ystep, nrows;
    float inv_proj[16], inv_view[16];
    uint32_t cam_const;
    float cam_near_rw, cam_far_rw;
    const float4_storage* tris;      // single layout, ntri * kTriFloat4
    const float4_storage* spheres;   // nsph
    uint32_t ntri, nsph;
    uint32_t ntx, nty, wt, stride;
    uint32_t* cull;                  // ntx * nty * stride words
};
constexpr uint32_t kCullTile = 8;
constexpr uint32_t kPixMaskMax = 1024;   // kparams::pmask: masks for triangle lists of up to this many entries
constexpr uint32_t kAnyMaxEntries = 512; // iqpt_anyhit_kernel: lists of up to this many (16 mask words in registers)

// Pixel state (accumulator, BGRA, RNG planes) is stored TILE-MAJOR over the owned set: 8x8 tiles
// of (column, owned row) in row-major tile order, pixels row-major inside a tile; tiles of the last
// tile column / row are narrower / shorter. A work-queue chunk is one tile, so a wave's loads and
// stores of pixel state are contiguous. The C ABI converts to the compact row-major order on the
// way in and out (iqpt_read, iqpt_read_rng, iqpt_copy_accum_device, checkpoints).
__host__ __device__ inline uint32_t tile_store_index(uint32_t col, uint32_t row, uint32_t ncols, uint32_t nrows) {
    const uint32_t tx = col / kCullTile, ty = row / kCullTile;
    const uint32_t th = nrows - ty * kCullTile < kCullTile ? nrows - ty * kCullTile : kCullTile;
    const uint32_t tw = ncols - tx * kCullTile < kCullTile ? ncols - tx * kCullTile : kCullTile;
    return ty * kCullTile * ncols + tx * kCullTile * th + (row % kCullTile) * tw + col % kCullTile;
}
__host__ __device__ inline void tile_decode(uint32_t s, uint32_t ncols, uint32_t nrows, uint32_t* col, uint32_t* row) {
    const uint32_t ty = s / (kCullTile * ncols);
    const uint32_t rem = s - ty * kCullTile * ncols;
    const uint32_t th = nrows - ty * kCullTile < kCullTile ? nrows - ty * kCullTile : kCullTile;
    const uint32_t tx = rem / (kCullTile * th);
    const uint32_t w = rem - tx * kCullTile * th;
    const uint32_t tw = ncols - tx * kCullTile < kCullTile ? ncols - tx * kCullTile : kCullTile;
    *col = tx * kCullTile + w % tw;
    *row = ty * kCullTile + w / tw;
}

// The BGRA8 frame is stored in COMPACT row-major order over the owned set (round 5), unlike the other pixel
// planes: nothing reads it on the device, so its readbacks need no reorder and a pipelined launch's frame buffer
// is the multi-GPU gather's send buffer as it is. A kernel writes pixel s (tile-major storage
// index) at tile_to_compact(s).
__host__ __device__ inline uint32_t tile_to_compact(uint32_t s, uint32_t ncols, uint32_t nrows) {
    uint32_t col, row;
    tile_decode(s, ncols, nrows, &col, &row);
    return row * ncols + col;
}

// Kernel option bits (all exact: each shortcut reproduces the reference's bits, see the kernel).
constexpr int kOptCamConst = 1 << 0;   // launch-constant 1/w of the inverse projection
constexpr int kOptAccTable = 1 << 1;   // running-mean 1/n, (n-1)/n table; c in {0,1} without a division
constexpr int kOptPair = 1 << 2;       // packed two-primitive intersection (pair layout)
constexpr int kOptLB5 = 1 << 3;        // __launch_bounds__ min 5 waves/SIMD (<= 96 VGPRs)
constexpr int kOptLB6 = 1 << 4;        // __launch_bounds__ min 6 waves/SIMD (<= 80 VGPRs)
constexpr int kOptSinCos = 1 << 5;     // shared reduction for cos(phi), sin(phi)
constexpr int kOptBranchless = 1 << 6; // pair MT without early exits (small resident scenes)
constexpr int kOptStats = 1 << 7;      // wave-level counters (diagnostic builds)
constexpr int kOptFastDiv = 1 << 8;    // short exact reciprocal / division forms (iq_fastdiv.h)
constexpr int kOptCull = 1 << 9;       // camera rays test only the pairs of their tile's mask (pair layout)
constexpr int kOptMaterials = 1 << 10; // per-primitive material table (RGB scatter records)
constexpr int kOptBvh = 1 << 11;       // secondary rays traverse the exact BVH (streamed scenes; inert
                                       // when the packet has none)
constexpr int kOptBvhPrimary = 1 << 12; // camera rays take the BVH too (instead of the tile masks)
constexpr int kOptCamAxis = 1 << 14;   // short camera transform for pitch-only cameras (kparams::cam_ax; the runtime
                                       // checks the zero pattern and the frame-wide normalization bounds)
constexpr int kOptSplit = 1 << 16;     // sample-parallel chains: speculative runs + anchored lanes (kparams::split_round)
constexpr int kOptScatter2 = 1 << 18;  // Oren–Nayar scatter with packed, branch-free transcendental pairs (iq_fp2.h)
constexpr int kOptPrio = 1 << 17;      // VALU issue priority for waves on the launch's critical path (no effect on results)
constexpr int kOptOverlap = 1 << 19;   // tiles bound to XCDs, launches overlap through per-tile completion counts
constexpr int kOptAnyHit = 1 << 20;    // streamed any-hit scenes (kparams::anyhit): BVH and list loops leave at the first
                                       // accepted triangle; its own variants, so other streamed scenes keep the registers
constexpr int kOptPipe = 1 << 21;      // resident scenes: a lane traces its path's ray and its next sample's camera ray in one
                                       // iteration; its own variants (4 waves/SIMD)
constexpr int kOptDefault = kOptCamConst | kOptAccTable | kOptPair | kOptSinCos | kOptLB5 | kOptFastDiv | kOptCull |
                            kOptBvh | kOptScatter2;
constexpr uint32_t kStatsHeader = 24;        // kOptStats: 24 counters, then per-wave (start, end, iterations)
constexpr uint32_t kStatsWaveSlots = 65536;
constexpr uint32_t kStatsQueueSlots = 65536;   // kOptStats: then the s_memrealtime at which queue position q was taken
constexpr uint32_t kStatsPhaseWords = 4;       // kOptStats: then per wave slot the shader-clock cycles (s_memtime) spent in
                                               // the closest hits, the shading, the next rays and the rest of the loop
constexpr uint32_t kAccTableMax = 1024;  // spp per launch covered by the LDS table (8 KiB)

// Launch wrappers (iqpt_kernels.hip). Return a hipError_t as int.
int launch_rng_init(void* stream, uint32_t width, uint32_t x0, uint32_t ncols, uint32_t y0,
                    uint32_t ystep, uint32_t nrows, uint64_t seed, const uint32_t* tables,
                    uint32_t* rng);
// Reorder `planes` planes of npix 32-bit words between tile-major storage and compact row-major
// order (to_compact: dst[compact] = src[storage]; else dst[storage] = src[compact]). `words` is the
// element width in 32-bit words (4 for the accumulator), the planes are npix * words apart.
int launch_relayout(void* stream, const uint32_t* src, uint32_t* dst, uint32_t ncols, uint32_t nrows,
                    uint32_t words, uint32_t planes, bool to_compact);
// Frame assembly after the multi-GPU gather: src = world blocks of `stride` pixels (rank r's rows base + r + k split
// in compact row-major order), dst = the W x H frame; `words` 32-bit words per pixel (1 BGRA8, 4 accumulator).
int launch_assemble_rows(void* stream, const uint32_t* src, uint32_t* dst, uint32_t width, uint32_t height,
                         uint32_t world, uint32_t split, uint32_t base, uint64_t stride, uint32_t words);
// Tile masks for kOptCull (one thread per tile word).
int launch_bin(void* stream, const kbin& b);
// Per-tile candidate counts from the masks (triangle pairs, sphere pairs), and the candidate lists.
// per tile of the masks: the certain flags of kparams::certain (one thread per tile)
int launch_certain(void* stream, const kbin& b, uint32_t* certain);
int launch_tile_count(void* stream, const uint32_t* cull, uint32_t ntiles, uint32_t wt, uint32_t stride,
                      uint32_t* cnt_tri, uint32_t* cnt_sph);
int launch_tile_list(void* stream, const uint32_t* cull, uint32_t ntiles, uint32_t wt, uint32_t stride,
                     const uint32_t* off_tri, const uint32_t* off_sph, uint32_t* list);
// Any-hit scenes: each tile's triangle candidate list reordered by how many of the tile's central rays a pair hits
// (any order gives the same bits there; the candidate-list loop leaves sooner)
int launch_tile_list_order(void* stream, const kbin& b, const uint32_t* off_tri, uint32_t* list);
int launch_pixel_mask(void* stream, const kbin& b, const uint32_t* off_tri, const uint32_t* list,
                      const uint32_t* pmask_off, uint32_t* pmask, uint32_t* certain);
// Device probe of the camera transforms (iqpt_debug_camera_rays): general and kOptCamAxis forms.
int launch_camera_probe(void* stream, const kparams& p, const float* ndc, float* gen, float* axis, uint32_t n,
                        bool do_axis);
// Test only: `blocks` blocks, each filling lds_bytes of LDS with a pattern (iqpt_debug_poison_lds).
int launch_lds_poison(void* stream, uint32_t pattern, uint32_t lds_bytes, uint32_t blocks);
// Device probe of the shared math (iqpt_debug_libm).
int launch_libm(void* stream, int fn, const float* a, const float* b, float* out, uint32_t n);
// grid_blocks = persistent grid size; lds_bytes dynamic LDS; stream = hipStream_t; opt = kOpt* mask.
int launch_render(void* stream, const kparams& p, uint32_t grid_blocks, uint32_t lds_bytes, bool stream_batches,
                  int opt);
// Max resident blocks per CU of the render kernel for the given dynamic LDS (occupancy query).
int render_occupancy(int max_depth, bool stream_batches, int opt, uint32_t lds_bytes, int* blocks_per_cu);
// kOptSplit: the windows, run states and run chunks before round 1, the stitch after it (fastdiv:
// the running mean's short division, as the render variant that produced the slots).
int launch_split_prep(void* stream, const ksplit& s);
int launch_split_stitch(void* stream, const ksplit& s, bool fastdiv);
bool render_variant_exists(int max_depth, bool stream_batches, int opt);
// Slot-parallel sphere pixels: resident scene, reference materials, max_depth <= 16,
// spp <= kAccTableMax.
bool spec_variant_exists(int max_depth, int opt);
uint32_t spec_lds(const kparams& p, const kspec& s);
int launch_spec(void* stream, const kparams& p, const kspec& s, int opt);
// resident iqpt_spec_kernel blocks per CU for this launch
int spec_occupancy(const kparams& p, const kspec& s, int opt, int* blocks);
// Certain-miss pixels (iqpt_sky_kernel): the p.miss pixels of `ntiles` tiles (tiles[i]),
// lane = pixel, one wave per tile; resident scenes, reference materials, spp <= kAccTableMax.
bool sky_variant_exists(int opt);
bool anyhit_variant_exists(int opt);
int launch_anyhit(void* stream, const kparams& p, int opt);
int launch_sky(void* stream, const kparams& p, const uint32_t* tiles, uint32_t ntiles, int opt);
// Sample-parallel anchored tiles (iqpt_fan_kernel): one block per tile of
// p.tile_order[0 .. ntiles) — tiles without sphere candidates, reference materials, resident scene
// (p.cull set, p.cull_wt <= 16), spp <= kAccTableMax.
bool fan_variant_exists(int opt);
uint32_t fan_lds(const kparams& p);
int launch_fan(void* stream, const kparams& p, uint32_t ntiles, int opt);
// Events (hipEvent_t, either may be null) recorded by the dispatch of the next render / spec / fan / sky
// kernel this thread launches (hipExtLaunchKernel) rather than by marker packets of their own; a launch
// function that launches nothing leaves them bound — the caller unbinds (nullptr, nullptr).
void bind_launch_events(void* start, void* stop);
// the events bound to the next launch (and unbind them): a launch of several kernels binds them to its first and last
void take_launch_events(void** start, void** stop);
constexpr int kRenderBlock = 256;
constexpr uint32_t kQueueChunk = 64;
const char* render_kernel_name();

}  // namespace iqpt
