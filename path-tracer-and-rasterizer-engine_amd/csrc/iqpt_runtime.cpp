// iqpt_runtime.cpp — the C ABI of include/iqpt.h over HIP: render contexts, packet relayout,
// launches, readback, timing and errors.
//
// Replaces the CUDA side of path_tracer (IoniqRE/path_tracer.cu:48-164, 368-404) and the upload
// half of scene::build_packet / free_packet (IoniqRE/scene.cu:183-264).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "iq_bvh.hpp"
#include "iq_host_math.hpp"
#include "iq_interval.h"
#include "iq_xorwow.h"
#include "iqpt.h"
#include "iqpt_internal.hpp"

namespace iqpt {

namespace {
thread_local std::string g_last_error;

// LDS budget under which the whole scene stays resident per block (no barriers in the loop).
constexpr uint32_t kLdsResidentBytes = 32 * 1024;
// Batch sizes when the scene is streamed through LDS (pairs: 10 KB + 4 KB; with the table, mask
// slots and scatter stack a block stays under 32 KB, so 5 blocks fit a CU).
constexpr uint32_t kTriBatch = 256;   // primitives per LDS batch (128 pairs = 10 KB)
constexpr uint32_t kSphBatch = 256;
// kOptBvhPrimary launches leave the batch region unused and park 13 words of path state per thread there
static_assert((kTriBatch / 2) * kTriPairFloat4 * 16 + (kSphBatch / 2) * kSphPairFloat4 * 16 >= 13 * kRenderBlock * 4,
              "the BVH-primary path-state slots must fit the scene-batch region");
constexpr int kTuneLaunches = 4;     // timed launches before the camera-ray path is chosen (A, B, A, B)
// kOptSplit auto mode: split when the owned pixels are fewer than this many per resident lane
constexpr double kSplitAutoPixelsPerLane = 1.2;
// spec launches: AUTO takes them below this many owned pixels per resident lane of the
// plain kernel (C3 shares: N = 8 has 0.8, N = 4 1.6, N = 2 3.2; pipelined spec launches 0.27 / 0.47 / 0.87 ms
// per step through the gather against plain 0.95 / 1.0 / 0.91; N = 1, 6.3, stays plain; profiles/r03/
// split_share_run37.json, r03_share_v11.json, run49_share{2,4,8}_2.json)
constexpr double kSpecAutoPixelsPerLane = 4.0;
constexpr size_t kSplitResBudget = size_t(8) << 30;   // speculative results (bytes)

std::once_flag g_tables_once;
std::vector<uint32_t> g_tables;  // A^(2^(67+i)), i < 32

const std::vector<uint32_t>& xorwow_tables() {
    std::call_once(g_tables_once, [] {
        g_tables.resize(32 * IQ_XORWOW_MAT_WORDS);
        iq_xorwow_subseq_tables(g_tables.data(), 32);
    });
    return g_tables;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(IQPT_ERR_HIP, std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
}
}  // namespace

void set_last_error(const std::string& msg) { g_last_error = msg; }
int fail(int status, const std::string& msg) {
    g_last_error = msg;
    return status;
}

}  // namespace iqpt

#define IQPT_HIP(call)                                                  \
    do {                                                                \
        hipError_t e_ = (call);                                         \
        if (e_ != hipSuccess) return iqpt::hip_fail(e_, #call);         \
    } while (0)

using iqpt::float4_storage;

struct iqpt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t width = 0, height = 0;
    iqpt_pixel_set set{};
    uint32_t ncols = 0, npix = 0;
    uint64_t seed = 0;
    int max_depth = 0;
    uint64_t frame = 0;
    int num_cus = 0;
    int num_xcc = 0;              // XCDs of the device (overlapped launches bind tiles to the 8 XCDs)
    uint32_t lds_per_block = 0;   // the device's LDS limit per workgroup (bytes)
    int opt = iqpt::kOptDefault;
    bool have_camera = false, have_packet = false;
    iqpt_camera cam{};
    // pixel state (compact over the owned set)
    float4_storage* d_lin = nullptr;
    uint32_t* d_bgra = nullptr;
    uint32_t* d_rng = nullptr;
    unsigned long long* d_rays = nullptr;
    uint32_t* d_queue = nullptr;
    unsigned long long* d_stats = nullptr;   // kOptStats counters (diagnostic variants)
    // scene (world space)
    float4_storage* d_tris = nullptr;
    float4_storage* d_tri_pairs = nullptr;
    float4_storage* d_tri_shade = nullptr;
    float4_storage* d_sph = nullptr;
    float4_storage* d_sph_pairs = nullptr;
    uint32_t ntri = 0, nsph = 0;
    std::vector<float4_storage> h_sph;   // world-space spheres (host copy: per-pixel sphere bundles, build_split)
    // material table (§8f.3), null without one
    uint32_t* d_tri_mat = nullptr;
    uint32_t* d_sph_mat = nullptr;
    float4_storage* d_mats = nullptr;
    // exact BVH for secondary rays (iq_bvh.hpp), null when the packet has few triangles
    float4_storage* d_bvh_nodes = nullptr;
    float4_storage* d_bvh_pairs = nullptr;
    uint32_t* d_bvh_always = nullptr;
    uint32_t bvh_nnodes = 0, bvh_nalways = 0;
    float bvh_md = 0.0f, bvh_gulp = 0.0f;
    // exact sphere BVH (iq_bvh.hpp), null when the packet has few spheres
    float4_storage* d_sbvh_nodes = nullptr;
    float4_storage* d_sbvh_sph = nullptr;
    uint32_t* d_sbvh_idx = nullptr;
    uint32_t* d_sbvh_always = nullptr;
    uint32_t sbvh_nnodes = 0, sbvh_nalways = 0;
    float sbvh_gulp = 0.0f;
    bool fast_rcp_ok = true;   // packet within the range of the kOptFastDiv reciprocals (upload)
    // kOptCull tile masks (iq_interval.h), rebuilt on the stream after a camera or packet change
    uint32_t* d_cull = nullptr;
    uint32_t* d_certain = nullptr;      // per tile: 64-bit mask of pixels certain to end on an emissive triangle
    bool certain_valid = false;         // d_certain holds the current masks' flags (no material table)
    bool certain_on = true;             // iqpt_debug_set_certain (A/B: 0 renders certain tiles normally)
    // certain-miss pixels: the tiles holding some (d_certain + 2 ntiles has their masks), the
    // pixel count; plain launches hand them to iqpt_sky_kernel (iqpt_debug_set_sky: 0 traces them as before)
    uint32_t* d_sky_tiles = nullptr;
    uint32_t n_sky_tiles = 0, n_sky_pixels = 0;
    bool sky_on = true;
    bool sky_active = false;            // the masks' miss pixels are the sky kernel's: the fan lists exclude them
    std::vector<uint64_t> h_miss;       // per tile: the certain-miss mask (host copy, for the fan lists)
    hipEvent_t ev_sky = nullptr;        // after the last sky kernel (the next one, maybe on the other stream, waits)
    hipStream_t sky_last = nullptr;     // the stream of the last sky kernel since the streams were joined
    uint32_t* d_tile_order = nullptr;   // work-queue order over tiles, built with the masks
    uint32_t* d_list = nullptr;         // candidate lists of the masks, then their offsets (tri, sph)
    uint64_t list_total = 0;
    uint32_t* d_pmask = nullptr;        // per-tile word offsets (ntiles + 1), the per-pixel candidate masks (kparams::pmask),
                                        // then 2 words per tile of certain pixels (kparams::pmask_certain)
    int pmask_mode = 2;                 // iqpt_debug_set_pixel_masks: 0 none, 1 in the plain kernel, 2 + iqpt_anyhit_kernel
    uint32_t pmask_tiles = 0;           // tiles with masks (a triangle list of 1 .. kPixMaskMax entries)
    uint64_t pmask_words = 0;           // mask words after the offsets
    bool pmask_all = false;             // every list within kAnyMaxEntries and no tile with a sphere candidate
    uint32_t list_max = 0;              // the longest triangle list
    bool last_anyk = false;             // the last launch ran iqpt_anyhit_kernel
    size_t cull_cap = 0;       // words allocated
    bool cull_valid = false;
    uint32_t cull_ntx = 0, cull_nty = 0, cull_wt = 0, cull_stride = 0;
    // timing
    struct timed_launch { hipEvent_t e0, e1, e1b; };   // e1b: the second stream's end (pipelined spec), or null
    std::vector<timed_launch> timed;
    std::vector<hipEvent_t> event_pool;
    // camera rays of a streamed scene with a BVH: tile masks or the BVH (kOptBvhPrimary), whichever
    // the first two launches after a packet upload time faster per sample (results are identical);
    // tools/ab_kernel.py fixes the option set instead (opt_fixed)
    bool opt_fixed = false;
    // stages 0..kTuneLaunches-1 time masks (even) and the BVH (odd) alternately; stage kTuneLaunches
    // decides on the fastest launch of each; reset by a packet upload or a camera change
    int tune_stage = 0;
    bool tune_primary = false;
    hipEvent_t tune_ev[2 * 4] = {};
    int last_opt = -1;           // option set of the last render launch (iqpt_debug_last_options)
    bool last_xcd_lists = false; // the last launch dealt its tiles to per-XCD lists (overlapped or streamed)
    // kOptSplit, sample-parallel chains: mode (IQPT_SPLIT_*), the split set built with
    // the masks (tiles whose camera rays may scatter), per-slot buffers sized for the launch
    int split_mode = IQPT_SPLIT_AUTO;
    bool split_last = false;     // the last launch ran split
    uint32_t n_split_tiles = 0, n_anchor = 0;
    uint32_t* d_split = nullptr;        // anchor_order[n_anchor], split_tiles[nst], sp_pix, sp_win, sp_rho,
                                        // left (ns_cap each)
    uint32_t* d_sp_st = nullptr;        // 6 x ns_cap
    uint32_t* d_run_st = nullptr;       // (g_max + 1) x 6 x ns_cap
    uint32_t* d_chunks = nullptr;       // 2 x g_max x split tiles: round-1 run chunks
    float4_storage* d_sp_acc = nullptr; // ns_cap
    float4_storage* d_res = nullptr;    // m_cap x ns_cap
    uint8_t* d_nres = nullptr;          // ns_cap x m_cap
    uint32_t split_refill_min = 16;     // idle lanes before a refill in split launches
    uint32_t stream_refill_min = 64;    // ... in streamed launches: whole waves (iqpt_debug_set_stream_refill)
    uint32_t resident_refill_min = 1;   // ... in resident plain launches (iqpt_debug_set_resident_refill)
    uint32_t split_heavy_rho = iqpt::kSplitHeavyRho;
    bool split_all_tiles = false;       // every tile in the split set (wall tiles: one slot per sample)
    bool fan_last = false;              // the last launch ran the anchored tiles in iqpt_fan_kernel
    // spec launches with the fan kernel: the pixels of split tiles whose own camera-ray
    // bundle may reach a sphere (the spec kernel's pixel list, "chain pixels"), and the fan kernel's tiles with
    // the lanes it owns (anchored tiles whole; split tiles without their sphere pixels)
    uint32_t* d_chain_pix = nullptr;
    uint32_t n_chain_pix = 0;
    uint32_t* d_fan_tiles = nullptr;
    uint64_t* d_fan_lanes = nullptr;
    uint32_t n_fan_tiles = 0;
    // spec launches: per sphere pixel (d_chain_pix) the last window, the chain's slots per
    // sample (history, zeroed when the pixel list changes), the slot colours; sized for (spec_n, spec_mcap)
    uint32_t* d_spec = nullptr;         // m, rho (spec_n each), run_count (2)
    float4_storage* d_spec_res = nullptr;
    uint32_t spec_n = 0, spec_mcap = 0;
    bool spec_rho_valid = false;
    bool spec_last = false;
    uint32_t spec_rho0 = iqpt::kSpecRho0;   // window of a pixel without history (iqpt_debug_set_spec)
    uint32_t spec_parity_rho = iqpt::kSpecParityRho;   // parity pixels' threshold (iqpt_debug_set_spec_parity; 0 off)
    uint32_t spec_parity_hi = iqpt::kSpecParityHi;     // ... and upper bound
    bool anyhit_on = true;                  // any-hit queries in triangle-only scenes (iqpt_debug_set_anyhit)
    bool pipe_on = true;                    // two rays per lane in resident plain launches (kOptPipe, iqpt_debug_set_two_ray)
    uint32_t spec_margin_div = 16;          // window margin: 1/16 of the extra slots, at least 4 (iqpt_debug_set_spec;
                                            // against 1/4, 5 % of the chains take a second round instead of 0.6 %,
                                            // yet -4 % per launch at N = 2 / 4 / 8, profiles/r03/spec_margins.json)
    // spec launches (iqpt_debug_set_specfan): 0 the two kernels on two streams, pipelined (the default), 1 one
    // after the other on one stream (measurement)
    int specfan_mode = 0;
    // spec plan: the sphere pixels ordered by their last chain's work, heaviest first, the
    // heavy ones with 32 or 64 lanes; built on the host from an asynchronous read of the history (performance
    // only: every plan gives the same bits). iqpt_debug_spec_plan: 0 off, 1 asynchronous (default), 2..5
    // synchronous before every launch (tests; 3, 4: every pixel 32 / 64 lanes, 5: mixed)
    int spec_plan_mode = 1;
    double spec_cap = 0.97;                 // a plan's lanes: this fraction of the resident lanes
    uint32_t* h_spec_rho = nullptr;      // pinned: the history read back (spec_n)
    uint32_t* h_spec_plan = nullptr;     // pinned: staging of the plan (3 spec_n)
    hipEvent_t ev_spec_rho = nullptr, ev_spec_plan = nullptr;
    bool spec_rho_pending = false;       // a history read in flight
    bool spec_plan_up = false;           // a plan upload was enqueued (ev_spec_plan)
    uint32_t* d_spec_plan = nullptr;     // order (spec_n words), then 2 words per block
    uint32_t spec_plan_n = 0;            // pixels of the plan (0: none; must equal n_chain_pix to be used)
    uint32_t spec_plan_blocks = 0;
    uint32_t spec_plan_age = 0;          // launches since the plan was built
    // Pipelined spec and fan launches: the spec kernel (or, FAN, the plain kernel over the
    // split tiles) on `stream`, the fan kernel on `stream2`, and no join at the end of a launch — launch
    // k + 1's pixels on `stream` follow launch k's there, its fan pixels launch k's on `stream2` (the two sets
    // are disjoint and the same for launches of one kind), so the fan stream runs ahead into the other's tail. Every other entry point joins (join_streams). Frame copies (iqpt_copy_frame_device_async)
    // go on `stream3` behind both kernels; from the first such copy on, launches write the two frame buffers
    // in turn and a launch waits only for the copy that read its buffer two launches earlier.
    bool pipe = false;                   // the last launch was pipelined and nothing has joined since
    int pipe_kind = 0;                   // ... a spec launch (1)
    hipStream_t stream3 = nullptr;
    hipEvent_t ev_pipe_end = nullptr;    // on `stream`, recorded by a copy behind a pipelined launch
    // the events the last pipelined launch's kernels recorded at their ends on `stream` / `stream2` (timing
    // events bound to the dispatches), or null: a copy behind the launch waits for them instead of recording
    // markers of its own
    hipEvent_t end1 = nullptr, end2 = nullptr;
    // copies behind pipelined launches (iqpt_copy_frame_device_async, the gather's send copy): from the first
    // one on, pipelined launches write a ring of kPipeRing frame buffers in turn (d_bgra points at the one
    // the last launch wrote). Copy s (1-based, copy_seq counts them) records pev[s % kPipeRing] on stream3
    // after reading its launch's buffer; pseq[b] is the last copy that read ring buffer b. A launch about
    // to write buffer b that a copy newer than pwaited read makes both render streams wait for copy
    // copy_seq - 2 (three launches back when every launch is copied: a copy still in flight is not waited
    // for), which stream3's order makes cover every buffer copied up to it: one wait per kPipeRing - 2
    // launches instead of one per launch (each wait is a packet on both streams between two kernels:
    // r04 run 21, 0.015-0.02 ms per share-8 step)
    uint32_t* d_pring[iqpt::kPipeRing] = {};
    hipEvent_t pev[iqpt::kPipeRing] = {};
    uint64_t pseq[iqpt::kPipeRing] = {};
    uint64_t copy_seq = 0, pwaited = 0;
    int pidx = 0;
    bool pring_on = false;
    uint32_t* d_bgra_own = nullptr;     // the allocations behind d_bgra / d_bgra_alt (views that swap)
    uint32_t* d_alt_own = nullptr;
    unsigned long long* d_spec_tl = nullptr;   // iqpt_debug_spec_timeline: per spec block timestamps
    size_t spec_tl_blocks = 0;
    bool spec_tl_on = false;
    size_t res_slots = 0;               // m_cap x ns_cap allocated (res, nres)
    double tune_work[4] = {0.0, 0.0, 0.0, 0.0};
    // kOptOverlap: consecutive render launches alternate between `stream` and
    // `stream2`, so launch k + 1 fills the CUs that launch k's tail leaves idle; it takes a tile only
    // when launch k has finished it (tile_done). Every other entry point joins the streams first.
    int overlap_mode = IQPT_OVERLAP_AUTO;
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_pre = nullptr;        // on `stream`, before its last overlapped launch
    hipEvent_t ev_s2 = nullptr;         // on `stream2`, after its last launch (join)
    bool s2_pending = false;            // stream2 has work `stream` has not waited for
    bool next_on_main = true;           // the next overlapped launch goes to `stream`
    bool ovl_zero = true;               // tile_done must be zeroed before the next overlapped launch
    uint32_t ovl_epoch = 0;             // overlapped launches since tile_done was zeroed
    uint32_t* d_tile_done = nullptr;    // ntiles
    uint32_t* d_xcd_order = nullptr;    // ntiles: XCD x's tiles at [xcd_off[x], xcd_off[x + 1])
    uint32_t xcd_off[9] = {};
    // streamed scenes (iqpt_debug_set_stream_xcd): 0 one queue over the cost order; 1 the per-XCD lists above
    // (a queue word per XCD: C5 -9 % at 1 spp per launch, where tiles are short and the one queue word is
    // contended; +0.2..1.4 % at 16 spp and C4 +4 % at 256, where the fixed lists end unevenly, r05 runs 38-39);
    // 2 per-XCD bands of kXcdBandRows tile rows dealt round-robin (each XCD's L2 sees a band at a time: +17 % at
    // 16 spp, the bands are not in cost order); 3 (default) 1 up to kStreamXcdMaxSpp samples per launch, else 0
    int stream_xcd = 3;
    uint32_t* d_xcd_band = nullptr;     // ntiles: XCD x's bands at [xcd_band_off[x], xcd_band_off[x + 1])
    uint32_t xcd_band_off[9] = {};
    uint32_t* d_ovl_err = nullptr;
    // stream-ordered frame copies across overlapped launches (iqpt_copy_frame_device_async): once the
    // first such copy is asked for, each overlapped launch writes the BGRA frame into the buffer the
    // previous launch did not (d_bgra is always the last written, d_bgra_alt the other), so launch k's
    // copy, queued on launch k's stream, reads a frame launch k + 1 never touches, and launch k + 2
    // (the same stream) writes it only after that copy
    uint32_t* d_bgra_alt = nullptr;
    hipStream_t last_ls = nullptr;      // the stream of the last render launch
    bool last_ovl = false;              // ... which was overlapped, and no call has joined the streams since
    double last_span_ms = 0.0;          // iqpt_kernel_time: first start to last end of the timed launches
    // forward-progress bounds of the kernels (iqpt_debug_set_limits lowers them in tests) and a bias added
    // to the per-tile wait targets of overlapped launches (tests: a wait that can never be satisfied)
    uint32_t spin_limit = iqpt::kOverlapSpinLimit, iter_limit = iqpt::kChainIterLimit, wait_bias = 0;
    // the kernels' error word, latched at the first synchronising call that sees it: after a wait that
    // gave up or a chain wave past its bound the pixel state is undefined, so every later call that
    // returns or persists pixel state fails until iqpt_checkpoint_load replaces the whole state
    uint32_t dev_err = 0;
    // multi-GPU frame delivery (iqpt_comm_init): an RCCL communicator over the ranks of one
    // frame's cyclic row split and its own stream. A gather copies the rank's pixels (compact order, padded
    // to comm_stride pixels) into one of kSendRing send buffers in turn — the copy of gather g waits only for
    // gather g - kSendRing — then ncclGather to the root, which assembles the frame from the rank blocks.
    void* comm = nullptr;                // ncclComm_t
    int comm_rank = 0, comm_world = 0;
    uint64_t comm_stride = 0;            // pixels per rank block: the most rows any rank owns x W
    hipStream_t cstream = nullptr;
    // send buffers in turn (the copy of gather g waits for gather g - kSendRing, long done: with two, a
    // gather slowed by the renders beside it held the next copies and, through them, the render streams)
    uint32_t* d_gsend[iqpt::kSendRing] = {};     // comm_stride x 4 words each
    hipEvent_t ev_gdone[iqpt::kSendRing] = {};   // on cstream, after the gather that read d_gsend[i]
    bool gdone_pend[iqpt::kSendRing] = {};
    uint32_t gpar = 0;                   // the send buffer of the next gather
    hipEvent_t ev_gcopy = nullptr;       // after the copy into the send buffer (cstream waits for it)
    hipEvent_t ev_gend = nullptr;        // on cstream, after the last gather (every other entry point joins it)
    bool comm_pend = false;
    uint32_t* d_grecv = nullptr;         // root: comm_world x comm_stride x 4 words
    uint32_t* d_gframe = nullptr;        // root: the assembled W x H x 4 words of iqpt_gather_read
    std::vector<std::pair<hipEvent_t, hipEvent_t>> gtimed;   // per gather: cstream events around it (iqpt_comm_time)
    // the gather's share of the CUs it runs beside (iqpt_debug_set_gather, before iqpt_comm_init): RCCL's
    // blocks per collective (ncclConfig_t::maxCTAs; 0: RCCL's choice) and cstream's priority (-1 lowest,
    // 0 the default, 1 highest)
    int gather_ctas = iqpt::kGatherCtas;
    int gather_prio = 0;
    int gather_skip = 0;                 // measurement only: 1 skips the collective, 2 the root's assembly,
                                         // 4 the render streams' waits for the frame copies
    bool timing_on = true;               // the launches' timing events (iqpt_debug_set_timing)
    bool sky_after = true;               // overlapped launches: the sky kernel behind the plain kernel (r04 run 35:
                                         // 0.988-0.992 -> 0.975-0.982 ms per C2 step)
};

namespace {

// Words of a BGRA8 frame buffer: the owned pixels, padded to the multi-GPU gather's block once a communicator
// exists (a pipelined launch's buffer is then the gather's send buffer itself)
size_t frame_words(const iqpt_ctx* c) {
    return std::max<size_t>((size_t)c->npix, (size_t)c->comm_stride);
}

int use_device(const iqpt_ctx* c) {
    IQPT_HIP(hipSetDevice(c->device));
    return IQPT_OK;
}

// kOptOverlap: make `stream` wait for the last launch on `stream2`; the next overlapped launch starts a
// new chain (tile_done zeroed on `stream`, no waits).
int join_streams(iqpt_ctx* c) {
    if (c->s2_pending) {
        IQPT_HIP(hipEventRecord(c->ev_s2, c->stream2));
        IQPT_HIP(hipStreamWaitEvent(c->stream, c->ev_s2, 0));
        c->s2_pending = false;
    }
    // pipelined launches: `stream` also waits for the frame copies still reading a frame buffer
    if (c->copy_seq > c->pwaited) {
        IQPT_HIP(hipStreamWaitEvent(c->stream, c->pev[c->copy_seq % iqpt::kPipeRing], 0));
        c->pwaited = c->copy_seq;
    }
    c->pipe = false;
    c->next_on_main = true;
    c->ovl_zero = true;
    c->last_ovl = false;
    c->sky_last = nullptr;             // everything before is ordered on `stream` now
    return IQPT_OK;
}

// Pipelined launches: the frame-copy stream and its two events, created when the first pipelined launch
// ends, so that iqpt_frame_stream names the stream the next copy goes on before any copy was asked for.
int ensure_copy_stream(iqpt_ctx* c) {
    if (!c->stream3 && hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        return iqpt::fail(IQPT_ERR_HIP, "frame copy stream");
    }
    return IQPT_OK;
}

// Every entry point but iqpt_render: the device, then the streams joined — the gathers in flight too
// (they read the send buffers and write the caller's frame; a render never waits for them: the copy
// into a send buffer is ordered behind the launch that wrote the frame, on the launch's own stream).
int enter(iqpt_ctx* c) {
    int st = use_device(c);
    if (st) return st;
    if (c->comm_pend) {
        IQPT_HIP(hipStreamWaitEvent(c->stream, c->ev_gend, 0));
        c->comm_pend = false;
    }
    return join_streams(c);
}

void cam_constants(const iqpt_camera& cam, uint32_t* is_const, float* near_rw, float* far_rw);

void free_scene(iqpt_ctx* c) {
    for (float4_storage** b : {&c->d_tris, &c->d_tri_pairs, &c->d_tri_shade, &c->d_sph, &c->d_sph_pairs, &c->d_mats,
                               &c->d_bvh_nodes, &c->d_bvh_pairs, &c->d_sbvh_nodes, &c->d_sbvh_sph}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    c->bvh_nnodes = c->bvh_nalways = 0;
    c->sbvh_nnodes = c->sbvh_nalways = 0;
    for (uint32_t** b : {&c->d_tri_mat, &c->d_sph_mat, &c->d_bvh_always, &c->d_sbvh_idx,
                         &c->d_sbvh_always}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    c->ntri = c->nsph = 0;
    c->cull_valid = false;
    c->tune_stage = 0;
    c->tune_primary = false;
}

void free_split(iqpt_ctx* c) {
    for (uint32_t** b : {&c->d_split, &c->d_sp_st, &c->d_run_st, &c->d_chunks}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    for (float4_storage** b : {&c->d_sp_acc, &c->d_res}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    if (c->d_nres) (void)hipFree(c->d_nres);
    c->d_nres = nullptr;
    for (uint32_t** b : {&c->d_chain_pix, &c->d_fan_tiles}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    if (c->d_fan_lanes) (void)hipFree(c->d_fan_lanes);
    c->d_fan_lanes = nullptr;
    c->n_chain_pix = c->n_fan_tiles = 0;
    c->spec_rho_valid = false;           // a new pixel list: no chain history, no plan
    c->spec_plan_n = 0;
    c->spec_rho_pending = false;
    c->n_split_tiles = c->n_anchor = 0;
    c->res_slots = 0;
}

// Chain launches with the fan kernel: which pixels of the split tiles can reach a sphere at all. The
// interval bundle of iq_interval.h (the same RN operation chain as the kernel's camera ray and sphere
// test, compiled for the host with contraction off) is evaluated per pixel over its jitter square: a
// pixel whose bundle rejects every sphere ends every sample on its first ray (every triangle is emissive
// under the reference's materials) and goes to the fan kernel with its tile's triangle mask; the rest
// are the chain kernel's. Without a material table and with at most 64 spheres (otherwise every pixel
// of a split tile stays with the chain kernel).
int build_pixel_split(iqpt_ctx* c, const std::vector<uint32_t>& anchor, const std::vector<uint32_t>& split,
                      const uint32_t* sp_pix) {
    // with the sky kernel on (sky_active), certain-miss pixels are its own: the fan kernel's lanes exclude them,
    // and tiles left with no lane leave its list
    std::vector<uint32_t> chain_pix, fan_tiles;
    std::vector<uint64_t> fan_lanes;
    const bool sky = c->sky_active && c->h_miss.size() == (size_t)c->cull_ntx * c->cull_nty;
    for (uint32_t t : anchor) {
        const uint64_t own = sky ? ~c->h_miss[t] : ~0ull;
        const uint32_t tx = t % c->cull_ntx, ty = t / c->cull_ntx;
        const uint32_t npt = std::min(iqpt::kCullTile, c->ncols - tx * iqpt::kCullTile) *
                             std::min(iqpt::kCullTile, c->set.nrows - ty * iqpt::kCullTile);
        if (own & (npt == 64u ? ~0ull : ((1ull << npt) - 1ull))) {
            fan_tiles.push_back(t);
            fan_lanes.push_back(own);
        }
    }
    const bool per_pixel = !c->d_mats && c->h_sph.size() == c->nsph && c->nsph <= 64;
    iqiv::camera_in ci;
    ci.width = c->width;
    ci.height = c->height;
    ci.rcp_width = 0.0f;
    ci.rcp_height = 0.0f;
    ci.inv_proj = c->cam.inv_proj;
    ci.inv_view = c->cam.inv_view;
    uint32_t cc = 0;
    cam_constants(c->cam, &cc, &ci.near_rw, &ci.far_rw);
    ci.cam_const = (int)cc;
    for (size_t st = 0; st < split.size(); ++st) {
        uint64_t lanes = 0;
        for (uint32_t i = 0; i < iqpt::kQueueChunk; ++i) {
            const uint32_t pix = sp_pix[st * iqpt::kQueueChunk + i];
            if (pix == ~0u) continue;
            // a certain miss is the sky kernel's whenever it runs (also without the per-pixel test below:
            // ADVICE r4, a resident scene of more than 64 spheres put them in the spec / chain list as well)
            if (sky && ((c->h_miss[split[st]] >> i) & 1ull)) continue;
            bool sphere = !per_pixel;
            if (per_pixel) {
                uint32_t col, row;
                iqpt::tile_decode(pix, c->ncols, c->set.nrows, &col, &row);
                const uint32_t x = c->set.x0 + col, y = c->set.y0 + row * c->set.ystep;
                const iqiv::bundle b = iqiv::camera_bundle(ci, x, x, y, y);
                for (uint32_t k = 0; k < c->nsph && !sphere; ++k) {
                    const float ctr[3] = {c->h_sph[k].x, c->h_sph[k].y, c->h_sph[k].z};
                    sphere = !(b.ok && iqiv::sphere_culled(b, ctr, c->h_sph[k].w));
                }
            }
            if (sphere) {
                chain_pix.push_back(pix);
            } else {
                lanes |= 1ull << i;
            }
        }
        if (sky) lanes &= ~c->h_miss[split[st]];
        if (lanes) {
            fan_tiles.push_back(split[st]);
            fan_lanes.push_back(lanes);
        }
    }
    if (!chain_pix.empty()) {
        if (hipMalloc(&c->d_chain_pix, chain_pix.size() * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "chain pixel list");
        IQPT_HIP(hipMemcpy(c->d_chain_pix, chain_pix.data(), chain_pix.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (!fan_tiles.empty()) {
        if (hipMalloc(&c->d_fan_tiles, fan_tiles.size() * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&c->d_fan_lanes, fan_lanes.size() * sizeof(uint64_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "fan tile list");
        IQPT_HIP(hipMemcpy(c->d_fan_tiles, fan_tiles.data(), fan_tiles.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        IQPT_HIP(hipMemcpy(c->d_fan_lanes, fan_lanes.data(), fan_lanes.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    }
    c->n_chain_pix = (uint32_t)chain_pix.size();
    c->n_fan_tiles = (uint32_t)fan_tiles.size();
    return IQPT_OK;
}

// The spec plan from the history rho (n sphere pixels) into h: the order (n words: pixel q
// at each position), then 2 words per block (first position, count | log2(lanes / 8) << 8); returns the
// block count. Work of pixel q: the slots of its window (spec_window of its last chain's slots per sample)
// times their mean length (those slots per sample again). Lanes per pixel (8, 16, 32 or 64) come from one
// per-lane work target E, the smallest whose lanes all fit the resident blocks (one block-wave; if even 8
// lanes each do not fit, E = total work / resident lanes): pixel q takes the fewest lanes with w_q / lanes
// <= E. Each block holds one lane class (256 lanes), pixels sorted by work per lane, and the blocks run
// heaviest per lane first, so the launch's longest block starts first and light blocks fill the tail.
uint32_t spec_build_plan(iqpt_ctx* c, const iqpt::kparams& p, const iqpt::kspec& ks, int opt, const uint32_t* rho,
                         uint32_t* h) {
    const uint32_t n = ks.n;
    std::vector<double> w(n);
    double total = 0.0, wmax = 0.0;
    for (uint32_t q = 0; q < n; ++q) {
        const uint32_t r = rho[q] ? rho[q] : ks.rho0;
        const uint32_t m = iqpt::spec_window(r, p.spp, ks.m_cap, ks.margin_div);
        // slots traced (the window's; a parity pixel's even ones and, expected, a quarter of the window's odd
        // ones in the pooled fix-up pass) times their mean length
        const bool parity = ks.parity_rho != 0u && r >= ks.parity_rho && r <= ks.parity_hi;
        w[q] = (double)m * (parity ? 0.625 : 1.0) * (double)std::max<uint32_t>(r, 256u) / 256.0;
        total += w[q];
        wmax = std::max(wmax, w[q]);
    }
    int occ = 0;
    if (iqpt::spec_occupancy(p, ks, opt, &occ) != 0 || occ < 1) occ = 1;
    const double cap = c->spec_cap * (double)c->num_cus * occ * 256.0;     // resident lanes, a little slack
    // lane classes: 256 / lanes pixels per block (a class that does not divide 256 leaves lanes idle); the
    // in-between classes let a plan use resident lanes that the next power of two would overfill (most
    // sphere pixels have the same work: r04 run 27)
    static constexpr uint32_t kLanes[iqpt::kSpecLaneClasses] = {8u, 16u, 32u, 64u};   // dividing 64: a pixel's
                                                                                           // lanes are one wave's
    constexpr uint8_t kTop = iqpt::kSpecLaneClasses - 1;
    auto cls_of = [&](uint32_t q, double e) -> uint8_t {
        uint8_t k = 0;
        while (k < kTop && w[q] > e * (double)kLanes[k]) ++k;
        return k;
    };
    auto lanes_at = [&](double e) {
        double sum = 0.0;
        for (uint32_t q = 0; q < n; ++q) sum += (double)kLanes[cls_of(q, e)];
        return sum;
    };
    double e = total / cap;                      // several block-waves: balanced work per lane
    if (lanes_at(wmax / 8.0) <= cap) {
        double lo = 0.0, hi = wmax / 8.0;        // lanes_at(hi) fits; find the smallest E that fits
        for (int it = 0; it < 40; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (lanes_at(mid) <= cap) hi = mid;
            else lo = mid;
        }
        e = hi;
    }
    std::vector<uint8_t> cls(n);
    double emax = 0.0;
    for (uint32_t q = 0; q < n; ++q) {
        uint8_t k = cls_of(q, e);
        if (c->spec_plan_mode == 3) k = 3;                                // 32 lanes
        if (c->spec_plan_mode == 4) k = kTop;                             // 64 lanes
        if (c->spec_plan_mode == 5) k = (uint8_t)(q % iqpt::kSpecLaneClasses);   // every class
        cls[q] = k;
        emax = std::max(emax, w[q] / (double)kLanes[k]);
    }
    // counting sort by (lane class, work per lane) descending
    constexpr uint32_t kB = 1024;
    constexpr uint32_t kC = iqpt::kSpecLaneClasses;
    std::vector<uint32_t> key(n), cnt((kC + 1) * kB + 2, 0);
    for (uint32_t q = 0; q < n; ++q) {
        const double pe = w[q] / (double)kLanes[cls[q]];
        const uint32_t b = emax > 0.0 ? std::min<uint32_t>(kB - 1, (uint32_t)(pe / emax * (kB - 1))) : 0u;
        key[q] = (kTop - cls[q]) * kB + (kB - 1 - b);   // ascending key: most lanes first, heaviest first
        cnt[key[q] + 1]++;
    }
    for (uint32_t k = 0; k < kC * kB + 1; ++k) cnt[k + 1] += cnt[k];
    for (uint32_t q = 0; q < n; ++q) h[cnt[key[q]]++] = q;
    // blocks of one class, then ordered by their first (heaviest) pixel's work per lane
    struct blk { double e; uint32_t first, word; };
    std::vector<blk> blocks;
    for (uint32_t i = 0; i < n;) {
        const uint32_t k = cls[h[i]], per = (uint32_t)iqpt::kSpecBlockLanes / kLanes[k];
        uint32_t m = 0;
        while (m < per && i + m < n && cls[h[i + m]] == k) ++m;
        blocks.push_back({w[h[i]] / (double)kLanes[k], i, m | (kLanes[k] << 8)});
        i += m;
    }
    std::stable_sort(blocks.begin(), blocks.end(), [](const blk& a, const blk& b) { return a.e > b.e; });
    for (size_t b = 0; b < blocks.size(); ++b) {
        h[n + 2 * b] = blocks[b].first;
        h[n + 2 * b + 1] = blocks[b].word;
    }
    return (uint32_t)blocks.size();
}

// The split set of kOptSplit: the tiles whose camera rays may scatter — a sphere
// candidate in the masks under the reference's materials (every triangle is emissive), any candidate
// with a material table — in queue order, and the other tiles' queue order. Slot sp of the split set
// is pixel sp % 64 of split tile sp / 64 (tile-major storage index, ~0u past a partial tile's end).
int build_split(iqpt_ctx* c, const std::vector<uint32_t>& order, const std::vector<uint32_t>& cnt) {
    free_split(c);
    const uint32_t ntiles = (uint32_t)order.size();
    std::vector<uint32_t> anchor, split;
    for (uint32_t t : order) {
        const bool scatters = c->split_all_tiles ||
                              (c->d_mats ? (cnt[t] + cnt[ntiles + t]) > 0 : cnt[ntiles + t] > 0);
        (scatters ? split : anchor).push_back(t);
    }
    if (anchor.empty() && split.empty()) return IQPT_OK;
    // (no split tile: the anchored list alone, for fan launches; every split launch needs split tiles)
    const size_t ns = split.size() * (size_t)iqpt::kQueueChunk;
    if (ns >= (1ull << 31)) return IQPT_OK;
    std::vector<uint32_t> host(anchor.size() + split.size() + 5 * ns, 0u);
    std::copy(anchor.begin(), anchor.end(), host.begin());
    std::copy(split.begin(), split.end(), host.begin() + anchor.size());
    uint32_t* sp_pix = host.data() + anchor.size() + split.size();
    for (size_t st = 0; st < split.size(); ++st) {
        const uint32_t t = split[st];
        const uint32_t tx = t % c->cull_ntx, ty = t / c->cull_ntx;
        const uint32_t th = std::min(iqpt::kCullTile, c->set.nrows - ty * iqpt::kCullTile);
        const uint32_t tw = std::min(iqpt::kCullTile, c->ncols - tx * iqpt::kCullTile);
        const uint32_t first = ty * iqpt::kCullTile * c->ncols + tx * iqpt::kCullTile * th;
        for (uint32_t i = 0; i < iqpt::kQueueChunk; ++i)
            sp_pix[st * iqpt::kQueueChunk + i] = i < tw * th ? first + i : ~0u;
    }
    if (hipMalloc(&c->d_split, host.size() * sizeof(uint32_t)) != hipSuccess ||
        (ns && hipMalloc(&c->d_sp_st, 6 * ns * sizeof(uint32_t)) != hipSuccess) ||
        (ns && hipMalloc(&c->d_sp_acc, ns * sizeof(float4_storage)) != hipSuccess)) {
        free_split(c);
        return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "split buffers");
    }
    IQPT_HIP(hipMemcpy(c->d_split, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    c->n_anchor = (uint32_t)anchor.size();
    c->n_split_tiles = (uint32_t)split.size();
    return build_pixel_split(c, anchor, split, sp_pix);
}

// (Re)build the kOptCull tile masks of the current camera and packet on the context's stream.
constexpr uint64_t kListBudget = 1ull << 26;   // candidate-list entries (256 MB)

int build_cull(iqpt_ctx* c) {
    const uint32_t ntp = (c->ntri + 1) / 2, nsp = (c->nsph + 1) / 2;
    c->cull_ntx = (c->ncols + iqpt::kCullTile - 1) / iqpt::kCullTile;
    c->cull_nty = (c->set.nrows + iqpt::kCullTile - 1) / iqpt::kCullTile;
    c->cull_wt = (ntp + 31) / 32;
    c->cull_stride = c->cull_wt + (nsp + 31) / 32;
    const size_t words = (size_t)c->cull_ntx * c->cull_nty * c->cull_stride;
    if (words == 0) {
        c->cull_valid = true;
        return IQPT_OK;
    }
    if (words > c->cull_cap) {
        if (c->d_cull) {
            IQPT_HIP(hipStreamSynchronize(c->stream));
            (void)hipFree(c->d_cull);
            c->d_cull = nullptr;
            c->cull_cap = 0;
        }
        if (hipMalloc(&c->d_cull, words * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "cull masks");
        c->cull_cap = words;
    }
    iqpt::kbin b;
    std::memset(&b, 0, sizeof b);
    b.width = c->width;
    b.height = c->height;
    b.x0 = c->set.x0;
    b.ncols = c->ncols;
    b.y0 = c->set.y0;
    b.ystep = c->set.ystep;
    b.nrows = c->set.nrows;
    std::memcpy(b.inv_proj, c->cam.inv_proj, sizeof b.inv_proj);
    std::memcpy(b.inv_view, c->cam.inv_view, sizeof b.inv_view);
    cam_constants(c->cam, &b.cam_const, &b.cam_near_rw, &b.cam_far_rw);
    b.tris = c->d_tris;
    b.spheres = c->d_sph;
    b.ntri = c->ntri;
    b.nsph = c->nsph;
    b.ntx = c->cull_ntx;
    b.nty = c->cull_nty;
    b.wt = c->cull_wt;
    b.stride = c->cull_stride;
    b.cull = c->d_cull;
    const int le = iqpt::launch_bin(c->stream, b);
    if (le != 0) return iqpt::hip_fail((hipError_t)le, "cull binning kernel");
    const uint32_t ntiles = c->cull_ntx * c->cull_nty;
    // certain pixels (iq_interval.h tri_certain): only under the reference's materials (every triangle
    // emissive) and for scenes resident in LDS. In a streamed scene a lane that leaves a certain pixel takes
    // a pixel of the next tile, so waves hold two tiles and their LDS batches test the union of both tiles'
    // candidates: C4 +66 % per launch whether the pixels are folded in the refill or by a kernel of their own
    // (profiles/r03/ab_certain.json, ab_streamed_certain_fold_rejected.json)
    // per tile: candidate triangle pairs and sphere pairs (the queue order's cost and the lists' sizes), read
    // back at once: the device buffer is freed before any later step can return early
    std::vector<uint32_t> cnt(2 * (size_t)ntiles);
    {
        uint32_t* d_cnt = nullptr;
        IQPT_HIP(hipMalloc(&d_cnt, 2 * (size_t)ntiles * sizeof(uint32_t)));
        const int lcnt = iqpt::launch_tile_count(c->stream, c->d_cull, ntiles, c->cull_wt, c->cull_stride, d_cnt,
                                                 d_cnt + ntiles);
        hipError_t e = lcnt ? (hipError_t)lcnt : hipMemcpyAsync(cnt.data(), d_cnt, cnt.size() * sizeof(uint32_t),
                                                                hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(d_cnt);
        if (e != hipSuccess) return iqpt::hip_fail(e, "tile counts");
    }
    c->certain_valid = false;
    c->sky_active = false;
    c->h_miss.clear();
    if (c->d_certain) (void)hipFree(c->d_certain);
    c->d_certain = nullptr;
    std::vector<uint32_t> certain;
    const uint64_t resident_bytes = (uint64_t)ntp * iqpt::kTriPairFloat4 * 16u + (uint64_t)nsp * iqpt::kSphPairFloat4 * 16u;
    if (c->d_sky_tiles) (void)hipFree(c->d_sky_tiles);
    c->d_sky_tiles = nullptr;
    c->n_sky_tiles = 0;
    c->n_sky_pixels = 0;
    // (resident scenes: streamed ones with certain pixels and the sky kernel — their BVH-primary variants, which
    // have no LDS batches — measured slower on C4 in round 5, 135 -> 161 ms)
    if (!c->d_mats && ntiles > 0 && resident_bytes <= iqpt::kLdsResidentBytes) {
        // per tile: the certain-hit mask (2 words), then after all tiles the certain-miss masks (2 words each)
        if (hipMalloc(&c->d_certain, 4 * (size_t)ntiles * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "certain pixel masks");
        const int lc = iqpt::launch_certain(c->stream, b, c->d_certain);
        if (lc != 0) return iqpt::hip_fail((hipError_t)lc, "certain pixel kernel");
        certain.resize(4 * (size_t)ntiles);
        IQPT_HIP(hipMemcpyAsync(certain.data(), c->d_certain, 4 * (size_t)ntiles * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                c->stream));
        IQPT_HIP(hipStreamSynchronize(c->stream));
        c->certain_valid = true;
        // the tiles holding certain-miss pixels: iqpt_sky_kernel's work list (one wave each)
        std::vector<uint32_t> sky;
        c->h_miss.assign(ntiles, 0ull);
        for (uint32_t t = 0; t < ntiles; ++t) {
            const uint64_t m = (uint64_t)certain[2 * (size_t)ntiles + 2 * (size_t)t] |
                               ((uint64_t)certain[2 * (size_t)ntiles + 2 * (size_t)t + 1] << 32);
            c->h_miss[t] = m;
            if (m) {
                sky.push_back(t);
                c->n_sky_pixels += (uint32_t)__builtin_popcountll(m);
            }
        }
        if (!sky.empty()) {
            if (hipMalloc(&c->d_sky_tiles, sky.size() * sizeof(uint32_t)) != hipSuccess)
                return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "sky tile list");
            IQPT_HIP(hipMemcpy(c->d_sky_tiles, sky.data(), sky.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
            c->n_sky_tiles = (uint32_t)sky.size();
        }
    }
    c->sky_active = c->sky_on && c->certain_on && c->certain_valid && c->n_sky_tiles > 0;
    if (!c->sky_active) c->h_miss.clear();
    // queue order over tiles (a queue chunk is one tile): most expensive first, so the pixels that set
    // the end of the launch are cheap ones. Cost = candidate triangle pairs + 8 x candidate sphere pairs
    // (a camera ray that can hit a sphere starts an Oren-Nayar path: more rays and the scatter shading).
    std::vector<uint32_t> cost(ntiles);
    for (uint32_t t = 0; t < ntiles; ++t) cost[t] = cnt[t] + 8u * cnt[ntiles + t];
    // a certain pixel costs a fold of its samples: a tile's cost scales with its uncertain pixels (fully
    // certain tiles last in the order)
    if (c->certain_valid && c->certain_on)
        for (uint32_t t = 0; t < ntiles; ++t) {
            const uint32_t tx = t % c->cull_ntx, ty = t / c->cull_ntx;
            const uint32_t npt = std::min(iqpt::kCullTile, c->ncols - tx * iqpt::kCullTile) *
                                 std::min(iqpt::kCullTile, c->set.nrows - ty * iqpt::kCullTile);
            uint32_t nc = (uint32_t)__builtin_popcountll((uint64_t)certain[2 * (size_t)t] |
                                                         ((uint64_t)certain[2 * (size_t)t + 1] << 32));
            // certain misses leave the plain kernel's work too when the sky kernel takes them
            if (c->sky_on)
                nc += (uint32_t)__builtin_popcountll((uint64_t)certain[2 * (size_t)ntiles + 2 * (size_t)t] |
                                                     ((uint64_t)certain[2 * (size_t)ntiles + 2 * (size_t)t + 1] << 32));
            cost[t] = (uint32_t)(((uint64_t)cost[t] * (npt - std::min(nc, npt)) + npt - 1) / npt);
        }
    // candidate lists for the streamed kernel (pairs of a tile without scanning its mask words): only
    // worth building where the masks are long; skipped when they would exceed the list budget
    if (c->d_list) (void)hipFree(c->d_list);
    c->d_list = nullptr;
    if (c->d_pmask) (void)hipFree(c->d_pmask);
    c->d_pmask = nullptr;
    c->pmask_tiles = 0;
    c->pmask_all = false;
    c->list_max = 0;
    const bool want_lists = c->cull_stride > 8;
    uint64_t total = 0;
    std::vector<uint32_t> off(2 * ((size_t)ntiles + 1));
    for (uint32_t t = 0; t < ntiles; ++t) {
        off[t] = (uint32_t)std::min<uint64_t>(total, 0xffffffffull);
        total += cnt[t];
    }
    off[ntiles] = (uint32_t)std::min<uint64_t>(total, 0xffffffffull);
    for (uint32_t t = 0; t < ntiles; ++t) {
        off[ntiles + 1 + t] = (uint32_t)std::min<uint64_t>(total, 0xffffffffull);
        total += cnt[ntiles + t];
    }
    off[2 * (size_t)ntiles + 1] = (uint32_t)std::min<uint64_t>(total, 0xffffffffull);
    if (want_lists && total > 0 && total <= kListBudget) {
        uint32_t* d_off = nullptr;
        bool ok = hipMalloc(&c->d_list, (total + off.size()) * sizeof(uint32_t)) == hipSuccess;
        if (ok) {
            d_off = c->d_list + total;
            ok = hipMemcpyAsync(d_off, off.data(), off.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                c->stream) == hipSuccess &&
                 iqpt::launch_tile_list(c->stream, c->d_cull, ntiles, c->cull_wt, c->cull_stride, d_off,
                                        d_off + ntiles + 1, c->d_list) == 0 &&
                 // any-hit scenes: the lists most-hit pairs first (the launch's loop leaves at the wave's last hit)
                 (!(c->nsph == 0 && !c->d_mats && c->anyhit_on) ||
                  iqpt::launch_tile_list_order(c->stream, b, d_off, c->d_list) == 0) &&
                 hipStreamSynchronize(c->stream) == hipSuccess;
        }
        if (!ok) {
            if (c->d_list) (void)hipFree(c->d_list);
            c->d_list = nullptr;
        } else {
            c->list_total = total;
            // per-pixel masks over the triangle lists (a miss ray near a silhouette walks only the entries its
            // own pixel may meet); without them (allocation or launch failure) the kernel walks whole lists
            // compact: 64 words per 32 entries of each tile with at most kPixMaskMax entries, after the offsets
            std::vector<uint32_t> pm_off((size_t)ntiles + 1);
            uint64_t pm_words = 0;
            for (uint32_t t = 0; t < ntiles; ++t) {
                pm_off[t] = (uint32_t)pm_words;          // (used only when every offset fits: `fits` below)
                if (cnt[t] <= iqpt::kPixMaskMax) pm_words += 64u * (((uint64_t)cnt[t] + 31u) / 32u);
            }
            pm_off[ntiles] = (uint32_t)pm_words;
            const bool fits = (uint64_t)ntiles + 1 + pm_words < 0xffffffffull;
            if (c->pmask_mode != 0 && fits &&
                hipMalloc(&c->d_pmask, ((size_t)ntiles + 1 + pm_words + 2 * (size_t)ntiles) * sizeof(uint32_t)) ==
                    hipSuccess &&
                !(hipMemcpyAsync(c->d_pmask, pm_off.data(), pm_off.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                 c->stream) == hipSuccess &&
                  iqpt::launch_pixel_mask(c->stream, b, d_off, c->d_list, c->d_pmask, c->d_pmask + ntiles + 1,
                                          c->d_pmask + ntiles + 1 + pm_words) == 0 &&
                  hipStreamSynchronize(c->stream) == hipSuccess)) {
                (void)hipFree(c->d_pmask);
                c->d_pmask = nullptr;
            }
            if (c->d_pmask) {
                c->pmask_words = pm_words;
                c->pmask_all = true;
                for (uint32_t t = 0; t < ntiles; ++t) {
                    c->list_max = std::max(c->list_max, cnt[t]);
                    c->pmask_tiles += (cnt[t] > 0 && cnt[t] <= iqpt::kPixMaskMax) ? 1u : 0u;
                    c->pmask_all = c->pmask_all && cnt[t] <= iqpt::kAnyMaxEntries && cnt[ntiles + t] == 0;
                }
            }
        }
    }
    std::vector<uint32_t> order(ntiles);
    for (uint32_t t = 0; t < ntiles; ++t) order[t] = t;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
    if (!c->d_tile_order && hipMalloc(&c->d_tile_order, (size_t)ntiles * sizeof(uint32_t)) != hipSuccess)
        return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "tile order");
    IQPT_HIP(hipMemcpy(c->d_tile_order, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    // kOptOverlap: the cost order dealt round-robin to the 8 XCDs (each list in cost order)
    {
        std::vector<uint32_t> xo;
        xo.reserve(ntiles);
        for (uint32_t x = 0; x < 8; ++x) {
            c->xcd_off[x] = (uint32_t)xo.size();
            for (uint32_t r = x; r < ntiles; r += 8) xo.push_back(order[r]);
        }
        c->xcd_off[8] = (uint32_t)xo.size();
        if (!c->d_xcd_order && hipMalloc(&c->d_xcd_order, (size_t)ntiles * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "XCD tile order");
        if (!c->d_tile_done && hipMalloc(&c->d_tile_done, (size_t)ntiles * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "tile completion counts");

        IQPT_HIP(hipMemcpy(c->d_xcd_order, xo.data(), xo.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        c->ovl_zero = true;
        // streamed scenes' bands: rows of tiles in bands of kXcdBandRows, band b to XCD b mod 8, in tile order
        constexpr uint32_t kXcdBandRows = 4;
        const uint32_t ntx = c->cull_ntx, nty = (ntiles + ntx - 1) / ntx;
        std::vector<uint32_t> xb;
        xb.reserve(ntiles);
        for (uint32_t x = 0; x < 8; ++x) {
            c->xcd_band_off[x] = (uint32_t)xb.size();
            for (uint32_t b = x; b * kXcdBandRows < nty; b += 8)
                for (uint32_t ty = b * kXcdBandRows; ty < std::min(nty, (b + 1) * kXcdBandRows); ++ty)
                    for (uint32_t tx = 0; tx < ntx; ++tx)
                        if (ty * ntx + tx < ntiles) xb.push_back(ty * ntx + tx);
        }
        c->xcd_band_off[8] = (uint32_t)xb.size();
        if (!c->d_xcd_band && hipMalloc(&c->d_xcd_band, (size_t)ntiles * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "XCD tile bands");
        IQPT_HIP(hipMemcpy(c->d_xcd_band, xb.data(), xb.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    c->split_last = false;
    int st = build_split(c, order, cnt);
    if (st != IQPT_OK) return st;
    c->cull_valid = true;
    return IQPT_OK;
}

// w of the unprojected near/far points is a launch constant when the perspective row of the
// inverse projection is (0, 0, m23, m33) with finite non-zero m23, m33 (camera_ray).
void cam_constants(const iqpt_camera& cam, uint32_t* is_const, float* near_rw, float* far_rw) {
    const float* P = cam.inv_proj;
    const float wf = P[11] + P[15];
    const bool fin = std::isfinite(P[11]) && std::isfinite(P[15]) && std::isfinite(wf);
    *is_const = 0;
    *near_rw = 0.0f;
    *far_rw = 0.0f;
    if (P[3] == 0.0f && P[7] == 0.0f && fin && P[11] != 0.0f && P[15] != 0.0f && wf != 0.0f) {
        *is_const = 1;
        *near_rw = 1.0f / P[15];
        *far_rw = 1.0f / wf;
    }
}

// kOptCamAxis (camera_ray_axis in iqpt_kernels.hip): the zero pattern of a pitch-only camera under a
// standard perspective inverse, no -0 among the chains' last addends, every entry finite,
// kOptCamConst's constant w, and — from the interval bundle of every camera ray of the frame
// (iq_interval.h) — normalize3's zero branch never taken and |far - near| < 2^100. Fills the 16
// launch constants; false when the camera does not qualify.
bool cam_axis_constants(const iqpt_camera& cam, float* k) {
    const float* P = cam.inv_proj;
    const float* V = cam.inv_view;
    for (int i = 0; i < 16; ++i)
        if (!std::isfinite(P[i]) || !std::isfinite(V[i])) return false;
    uint32_t cc = 0;
    float nrw = 0.0f, frw = 0.0f;
    cam_constants(cam, &cc, &nrw, &frw);
    if (!cc || !std::isfinite(nrw) || !std::isfinite(frw)) return false;
    for (int i : {1, 2, 4, 6, 8, 9})
        if (P[i] != 0.0f) return false;
    for (int i : {1, 2, 4, 8})
        if (V[i] != 0.0f) return false;
    for (float last : {P[12], P[13], P[14], V[12], V[13], V[14]})
        if (last == 0.0f && std::signbit(last)) return false;
    if (cam.width == 0 || cam.height == 0) return false;
    iqiv::camera_in ci;
    ci.width = cam.width;
    ci.height = cam.height;
    ci.rcp_width = 0.0f;
    ci.rcp_height = 0.0f;
    ci.inv_proj = P;
    ci.inv_view = V;
    ci.cam_const = 1;
    ci.near_rw = nrw;
    ci.far_rw = frw;
    const iqiv::bundle b = iqiv::camera_bundle(ci, 0, cam.width - 1, 0, cam.height - 1);
    if (!b.ok || !(b.len.hi < 0x1p100f)) return false;
    // unprojected z of the near / far point (camera_ndc's chain; its zero terms only change the
    // sign of a zero inner sum, which the last addend P[14] (not -0) absorbs), divided by w
    const float zn = (((0.0f + 0.0f) + 0.0f * P[10]) + P[14]) * nrw;
    const float zf = (((0.0f + 0.0f) + 1.0f * P[10]) + P[14]) * frw;
    const float vals[16] = {P[0], P[5], P[12], P[13], nrw, frw, V[0], V[12], V[5], V[6], V[13], V[14],
                            zn * V[9], zf * V[9], zn * V[10], zf * V[10]};
    for (int i = 0; i < 16; ++i) {
        if (!std::isfinite(vals[i])) return false;
        k[i] = vals[i];
    }
    return true;
}

// Exact BVH for secondary rays (iq_bvh.hpp) over the world-space triangles `tris` (kTriFloat4 each)
// and the spheres (for the scene box). Fills the host arrays the upload copies to the device.
struct bvh_host {
    std::vector<float4_storage> nodes, pairs;
    std::vector<uint32_t> always;
    float md, gulp;
};
constexpr uint32_t kBvhMinTriangles = 256;

bool build_bvh(const std::vector<float4_storage>& tris, const std::vector<float4_storage>& sph, bvh_host& out) {
    const size_t ntri = tris.size() / iqpt::kTriFloat4;
    if (ntri < kBvhMinTriangles) return false;
    // scene box (exact corners of every triangle in double, spheres' centre +- radius)
    double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    std::vector<double> corners(ntri * 9);
    for (size_t k = 0; k < ntri; ++k) {
        const float4_storage* t = &tris[k * iqpt::kTriFloat4];
        const double v0[3] = {t[0].x, t[0].y, t[0].z};
        const double e1[3] = {t[0].w, t[1].x, t[1].y}, e2[3] = {t[1].z, t[1].w, t[2].x};
        for (int a = 0; a < 3; ++a) {
            const double c3[3] = {v0[a], v0[a] + e1[a], v0[a] + e2[a]};
            for (int q = 0; q < 3; ++q) {
                corners[k * 9 + 3 * q + a] = c3[q];
                blo[a] = std::min(blo[a], c3[q]);
                bhi[a] = std::max(bhi[a], c3[q]);
            }
        }
    }
    for (const float4_storage& s4 : sph) {
        const double c[3] = {s4.x, s4.y, s4.z}, r = std::fabs((double)s4.w);
        for (int a = 0; a < 3; ++a) {
            blo[a] = std::min(blo[a], c[a] - r);
            bhi[a] = std::max(bhi[a], c[a] + r);
        }
    }
    double ext = 0.0, maxabs = 0.0;
    for (int a = 0; a < 3; ++a) {
        ext = std::max(ext, bhi[a] - blo[a]);
        maxabs = std::max({maxabs, std::fabs(blo[a]), std::fabs(bhi[a])});
    }
    if (!std::isfinite(ext) || maxabs > 1e9) return false;
    // rays may use the BVH with |d_i| <= md and a finite origin (the bound holds for any origin:
    // it grows with the origin's distance S to the node, iq_bvh.hpp)
    const double Md = 1.001;
    out.md = 1.001f;
    // a box side lo - g rounds to nearest: |error| <= 2^-24 (maxabs + g); the kernel adds gulp and
    // scales g by 1 + 2^-20, which covers it
    double gc_max = 0.0;
    iqbvh::build_input in;
    for (size_t k = 0; k < ntri; ++k) {
        const float4_storage* t = &tris[k * iqpt::kTriFloat4];
        const float e1[3] = {t[0].w, t[1].x, t[1].y}, e2[3] = {t[1].z, t[1].w, t[2].x};
        const iqbvh::tri_coeffs b = iqbvh::triangle_coeffs(e1, e2, Md);
        if (!b.eligible) {
            out.always.push_back((uint32_t)k);
            continue;
        }
        for (int a = 0; a < 3; ++a) {
            const double lo = std::min({corners[k * 9 + a], corners[k * 9 + 3 + a], corners[k * 9 + 6 + a]});
            const double hi = std::max({corners[k * 9 + a], corners[k * 9 + 3 + a], corners[k * 9 + 6 + a]});
            in.lo.push_back(iqbvh::round_down(lo));
            in.hi.push_back(iqbvh::round_up(hi));
            in.centroid.push_back((float)((lo + hi) * 0.5));
        }
        const double co[4] = {b.gR, b.gB, b.tA, b.tB};
        gc_max = std::max(gc_max, b.gC);
        for (double v : co) in.coeff.push_back(iqbvh::round_up(v));
        in.normal.push_back(iqbvh::triangle_normal(e1, e2, Md, b.edet));
        in.edet.push_back(b.edet);
        in.tris.push_back((uint32_t)k);
    }
    // the D-independent part of the growth (gC) is applied as one scene-wide maximum
    out.gulp = iqbvh::round_up(maxabs * 0x1p-22 + gc_max);
    iqbvh::build_output bo;
    iqbvh::build(in, bo);
    // the 64-byte device node (iqpt_internal.hpp kBvhNodeFloat4): a leaf's successor is always the next
    // node, so one word holds the link — skip pointer (inner) or 1 << 31 | first pair << 8 | count (leaf);
    // tA, tB as bf16 rounded up; the cone as A = Nmin cos(beta) (down) and B = Nmin sin(beta) (up), from
    // which the kernel bounds Nmin |d| cos(theta + beta) = |d| cos(theta) A - |d| sin(theta) B
    if (bo.order.size() / 2 >= (1u << 23)) return false;
    for (const iqbvh::node& n : bo.nodes) {
        const uint32_t link = n.first_count ? (0x80000000u | n.first_count) : n.skip;
        const uint32_t tab = (iqbvh::bf16_up_bits(n.tA) << 16) | iqbvh::bf16_up_bits(n.tB);
        float4_storage w[4] = {{n.bmin[0], n.bmin[1], n.bmin[2], 0.0f},
                               {n.bmax[0], n.bmax[1], n.bmax[2], 0.0f},
                               {n.axis[0], n.axis[1], n.axis[2], n.edet},
                               {n.gR, n.gB, 0.0f, 0.0f}};
        std::memcpy(&w[0].w, &link, 4);
        std::memcpy(&w[1].w, &tab, 4);
        if (n.cos_beta > 0.0f && n.nmin > 0.0f) {
            w[3].z = iqbvh::round_down((double)n.cos_beta * (double)n.nmin);
            w[3].w = iqbvh::round_up((double)n.sin_beta * (double)n.nmin);
        }
        for (const float4_storage& v : w) out.nodes.push_back(v);
    }
    // leaf pairs in the kernel's pair layout (iqpt_internal.hpp), padding elements zero; the two
    // packet indices ride in the record's spare last two words (no separate index load per pair)
    const size_t npairs = bo.order.size() / 2;
    out.pairs.assign(npairs * iqpt::kTriPairFloat4, float4_storage{0.0f, 0.0f, 0.0f, 0.0f});
    for (size_t q = 0; q < bo.order.size(); ++q) {
        std::memcpy(&out.pairs[(q / 2) * iqpt::kTriPairFloat4 + 4].z + (q & 1), &bo.order[q], 4);
        if (bo.order[q] == ~0u) continue;
        const float4_storage* t = &tris[(size_t)bo.order[q] * iqpt::kTriFloat4];
        const float f[9] = {t[0].x, t[0].y, t[0].z, t[0].w, t[1].x, t[1].y, t[1].z, t[1].w, t[2].x};
        float* dst = &out.pairs[(q / 2) * iqpt::kTriPairFloat4].x;
        for (int comp = 0; comp < 9; ++comp) dst[2 * comp + (q & 1)] = f[comp];
    }
    return true;
}

// Exact sphere BVH (iq_bvh.hpp) over the world-space spheres (center.xyz, radius): spheres much larger
// than the median stay on the always-tested list. None for few spheres or coordinates beyond 2^60.
struct sbvh_host {
    std::vector<float4_storage> nodes, sph;
    std::vector<uint32_t> idx, always;
    float gulp;
};
constexpr uint32_t kSbvhMinSpheres = 64;
constexpr size_t kSbvhMaxSpheres = size_t(1) << 24;

bool build_sbvh(const std::vector<float4_storage>& sph, sbvh_host& out) {
    const size_t n = sph.size();
    // a leaf packs first << 8 | count (iq_bvh.hpp build_spheres): indices must stay below 2^24
    if (n < kSbvhMinSpheres || n >= kSbvhMaxSpheres) return false;
    std::vector<float> s4(4 * n), radii(n);
    double maxabs = 0.0;
    for (size_t k = 0; k < n; ++k) {
        const float v[4] = {sph[k].x, sph[k].y, sph[k].z, sph[k].w};
        for (int a = 0; a < 4; ++a) {
            if (!std::isfinite(v[a]) || std::fabs(v[a]) > 0x1p60f) return false;
            s4[4 * k + a] = v[a];
        }
        radii[k] = std::fabs(v[3]);
        for (int a = 0; a < 3; ++a) maxabs = std::max(maxabs, std::fabs((double)v[a]) + std::fabs((double)v[3]));
    }
    std::vector<float> sorted(radii);
    std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
    const double big = 8.0 * (double)sorted[n / 2];
    std::vector<uint32_t> ids;
    for (size_t k = 0; k < n; ++k) {
        if ((double)radii[k] > big) out.always.push_back((uint32_t)k);
        else ids.push_back((uint32_t)k);
    }
    std::vector<iqbvh::sph_node> nodes;
    std::vector<uint32_t> order;
    iqbvh::build_spheres(s4, ids, nodes, order);
    for (const iqbvh::sph_node& nd : nodes) {
        float4_storage lo, hi;
        lo.x = nd.bmin[0];
        lo.y = nd.bmin[1];
        lo.z = nd.bmin[2];
        std::memcpy(&lo.w, &nd.skip, 4);
        hi.x = nd.bmax[0];
        hi.y = nd.bmax[1];
        hi.z = nd.bmax[2];
        std::memcpy(&hi.w, &nd.first_count, 4);
        out.nodes.push_back(lo);
        out.nodes.push_back(hi);
        out.nodes.push_back(float4_storage{nd.rmin, nd.rmax, 0.0f, 0.0f});
    }
    for (uint32_t k : order) out.sph.push_back(sph[k]);
    out.idx = order;
    // a grown box side lo - g rounds to nearest: |error| <= 2^-24 (maxabs + g), covered by gulp and
    // the kernel's (1 + 2^-16) on g
    out.gulp = iqbvh::round_up(maxabs * 0x1p-22);
    return true;
}

// Pixel-state planes between device tile-major storage and host compact row-major order
// (iqpt_internal.hpp): a device reorder into a temporary buffer plus one copy. Synchronises.
int fetch_compact(iqpt_ctx* c, const void* dev, uint32_t words, uint32_t planes, void* host) {
    const size_t bytes = (size_t)c->npix * words * planes * sizeof(uint32_t);
    if (bytes == 0) return IQPT_OK;
    void* tmp = nullptr;
    if (hipMalloc(&tmp, bytes) != hipSuccess) return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "readback buffer");
    hipError_t e = (hipError_t)iqpt::launch_relayout(c->stream, static_cast<const uint32_t*>(dev),
                                                      static_cast<uint32_t*>(tmp), c->ncols, c->set.nrows, words,
                                                      planes, true);
    if (e == hipSuccess) e = hipMemcpyAsync(host, tmp, bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(tmp);
    return e == hipSuccess ? IQPT_OK : iqpt::hip_fail(e, "readback");
}

int store_compact(iqpt_ctx* c, const void* host, uint32_t words, uint32_t planes, void* dev) {
    const size_t bytes = (size_t)c->npix * words * planes * sizeof(uint32_t);
    if (bytes == 0) return IQPT_OK;
    void* tmp = nullptr;
    if (hipMalloc(&tmp, bytes) != hipSuccess) return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "upload buffer");
    hipError_t e = hipMemcpyAsync(tmp, host, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = (hipError_t)iqpt::launch_relayout(c->stream, static_cast<const uint32_t*>(tmp), static_cast<uint32_t*>(dev),
                                              c->ncols, c->set.nrows, words, planes, false);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(tmp);
    return e == hipSuccess ? IQPT_OK : iqpt::hip_fail(e, "upload");
}

// The sum of the spread ray counters (iqpt_internal.hpp kRaySlots); the streams are synchronised.
int read_rays(iqpt_ctx* c, unsigned long long* total) {
    std::vector<unsigned long long> slots((size_t)iqpt::kRaySlots * iqpt::kRaySlotStride);
    IQPT_HIP(hipMemcpy(slots.data(), c->d_rays, slots.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long v = 0;
    for (uint32_t k = 0; k < iqpt::kRaySlots; ++k) v += slots[(size_t)k * iqpt::kRaySlotStride];
    *total = v;
    return IQPT_OK;
}

// After the context's streams are synchronised: read the kernels' error word and latch it (see
// iqpt_ctx::dev_err). Returns IQPT_ERR_HIP while an error is latched.
int check_dev_err(iqpt_ctx* c) {
    if (!c->dev_err) {
        uint32_t err = 0;
        IQPT_HIP(hipMemcpy(&err, c->d_ovl_err, sizeof err, hipMemcpyDeviceToHost));
        c->dev_err = err;
    }
    if (!c->dev_err) return IQPT_OK;
    return iqpt::fail(IQPT_ERR_HIP, std::string((c->dev_err & 4u) ? "launch: an XCD's tile list was never taken"
                                                                   : "overlapped launch: a per-tile wait timed out") +
                                        " (pixel state undefined until iqpt_checkpoint_load)");
}

hipEvent_t take_event(iqpt_ctx* c) {
    if (!c->timing_on) return nullptr;
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// RCCL, bound at the first iqpt_comm_* call (dlopen by SONAME): a process that already holds an RCCL — the
// one PyTorch-ROCm ships, also librccl.so.1 — shares it instead of loading a second copy, and a single-GPU
// user of libiqpt never needs it. The entry points are RCCL's C API (/opt/rocm/include/rccl/rccl.h).
struct rccl_api {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_init_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;   // optional
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    std::string why;
};

const rccl_api& rccl() {
    static rccl_api api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
        if (!h) {
            const char* e = dlerror();
            api.why = std::string("RCCL not loadable: ") + (e ? e : "librccl.so.1");
            return;
        }
        api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        api.comm_init_config = reinterpret_cast<decltype(api.comm_init_config)>(dlsym(h, "ncclCommInitRankConfig"));
        api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        api.gather = reinterpret_cast<decltype(api.gather)>(dlsym(h, "ncclGather"));
        api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
        if (!api.get_unique_id || !api.comm_init_rank || !api.comm_destroy || !api.gather || !api.error_string) {
            api.get_unique_id = nullptr;
            api.why = "RCCL lacks ncclGetUniqueId / ncclCommInitRank / ncclCommDestroy / ncclGather";
        }
    });
    return api;
}

int rccl_fail(ncclResult_t r, const char* what) {
    return iqpt::fail(IQPT_ERR_HIP, std::string(what) + ": " + (rccl().error_string ? rccl().error_string(r) : "?"));
}

void free_comm(iqpt_ctx* c) {
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->comm && rccl().comm_destroy) (void)rccl().comm_destroy(static_cast<ncclComm_t>(c->comm));
    c->comm = nullptr;
    for (int i = 0; i < iqpt::kSendRing; ++i) {
        if (c->d_gsend[i]) (void)hipFree(c->d_gsend[i]);
        c->d_gsend[i] = nullptr;
        if (c->ev_gdone[i]) (void)hipEventDestroy(c->ev_gdone[i]);
        c->ev_gdone[i] = nullptr;
        c->gdone_pend[i] = false;
    }
    for (uint32_t** b : {&c->d_grecv, &c->d_gframe}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    for (hipEvent_t* e : {&c->ev_gcopy, &c->ev_gend}) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
    }
    for (auto& g : c->gtimed) {
        c->event_pool.push_back(g.first);
        c->event_pool.push_back(g.second);
    }
    c->gtimed.clear();
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    c->cstream = nullptr;
    c->comm_pend = false;
    c->comm_world = 0;
}

}  // namespace

extern "C" {

int iqpt_abi_version(void) { return IQPT_ABI_VERSION; }

const char* iqpt_error_string(int status) {
    switch (status) {
    case IQPT_OK: return "IQPT_OK";
    case IQPT_ERR_INVALID_ARG: return "IQPT_ERR_INVALID_ARG";
    case IQPT_ERR_HIP: return "IQPT_ERR_HIP";
    case IQPT_ERR_OUT_OF_MEMORY: return "IQPT_ERR_OUT_OF_MEMORY";
    case IQPT_ERR_NO_DEVICE: return "IQPT_ERR_NO_DEVICE";
    case IQPT_ERR_NOT_READY: return "IQPT_ERR_NOT_READY";
    case IQPT_ERR_UNSUPPORTED: return "IQPT_ERR_UNSUPPORTED";
    default: return "IQPT_ERR_UNKNOWN";
    }
}

const char* iqpt_last_error(void) { return iqpt::g_last_error.c_str(); }

const char* iqpt_kernel_name(void) { return iqpt::render_kernel_name(); }

int iqpt_create(int device, uint32_t width, uint32_t height, const iqpt_pixel_set* pixels, uint64_t seed,
                int max_depth, iqpt_ctx** out) {
    if (!out) return iqpt::fail(IQPT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (width == 0 || height == 0 || width > 65535 || height > 65535)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "frame must be 1..65535 pixels per side (camera stores uint16)");
    if (max_depth < 1) return iqpt::fail(IQPT_ERR_INVALID_ARG, "max_depth must be >= 1");
    if (max_depth > IQPT_MAX_DEPTH_LIMIT)
        return iqpt::fail(IQPT_ERR_UNSUPPORTED, "max_depth above IQPT_MAX_DEPTH_LIMIT");
    iqpt_pixel_set ps = pixels ? *pixels : iqpt_pixel_set{0, width, 0, 1, height};
    if (ps.x1 <= ps.x0 || ps.x1 > width || ps.nrows == 0 || ps.ystep == 0 ||
        (uint64_t)ps.y0 + (uint64_t)(ps.nrows - 1) * ps.ystep >= height)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "pixel set outside the frame");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return iqpt::fail(IQPT_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= count) return iqpt::fail(IQPT_ERR_NO_DEVICE, "device index out of range");

    iqpt_ctx* c = new iqpt_ctx();
    c->device = device;
    c->width = width;
    c->height = height;
    c->set = ps;
    c->ncols = ps.x1 - ps.x0;
    c->npix = c->ncols * ps.nrows;
    c->seed = seed;
    c->max_depth = max_depth;
    auto cleanup = [&](int st) {
        iqpt_destroy(c);
        return st;
    };
    int st = use_device(c);
    if (st) return cleanup(st);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return cleanup(iqpt::fail(IQPT_ERR_HIP, "hipGetDeviceProperties"));
    c->num_cus = prop.multiProcessorCount;
    c->lds_per_block = (uint32_t)prop.sharedMemPerBlock;
    if (hipDeviceGetAttribute(&c->num_xcc, hipDeviceAttributeNumberOfXccs, device) != hipSuccess) {
        (void)hipGetLastError();
        c->num_xcc = 0;
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return cleanup(iqpt::fail(IQPT_ERR_HIP, "hipStreamCreate"));
    const size_t n = c->npix;
    if (hipMalloc(&c->d_lin, n * sizeof(float4_storage)) != hipSuccess ||
        hipMalloc(&c->d_bgra, n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->d_rng, 6 * n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->d_rays, iqpt::kRaySlots * iqpt::kRaySlotStride * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_queue, (4 + iqpt::kOverlapQueueWords) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->d_ovl_err, sizeof(uint32_t)) != hipSuccess)
        return cleanup(iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "device allocation of the frame state failed"));
    c->d_bgra_own = c->d_bgra;
    // path_tracer.cu:134-135: both buffers start at zero
    if (hipMemsetAsync(c->d_lin, 0, n * sizeof(float4_storage), c->stream) != hipSuccess ||
        hipMemsetAsync(c->d_bgra, 0, n * sizeof(uint32_t), c->stream) != hipSuccess ||
        hipMemsetAsync(c->d_rays, 0, iqpt::kRaySlots * iqpt::kRaySlotStride * sizeof(unsigned long long), c->stream) != hipSuccess ||
        hipMemsetAsync(c->d_ovl_err, 0, sizeof(uint32_t), c->stream) != hipSuccess)
        return cleanup(iqpt::fail(IQPT_ERR_HIP, "hipMemsetAsync"));
    // renderer_init_kernel (path_tracer.cu:139): curand_init(seed, pixelid, 0)
    const std::vector<uint32_t>& tables = iqpt::xorwow_tables();
    uint32_t* d_tables = nullptr;
    if (hipMalloc(&d_tables, tables.size() * sizeof(uint32_t)) != hipSuccess)
        return cleanup(iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "jump tables"));
    hipError_t e = hipMemcpyAsync(d_tables, tables.data(), tables.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream);
    int lst = e == hipSuccess ? iqpt::launch_rng_init(c->stream, width, ps.x0, c->ncols, ps.y0, ps.ystep, ps.nrows,
                                                      seed, d_tables, c->d_rng)
                              : (int)e;
    hipError_t se = hipStreamSynchronize(c->stream);
    (void)hipFree(d_tables);
    if (lst != 0) return cleanup(iqpt::hip_fail((hipError_t)lst, "rng init kernel"));
    if (se != hipSuccess) return cleanup(iqpt::hip_fail(se, "rng init sync"));
    *out = c;
    return IQPT_OK;
}

int iqpt_destroy(iqpt_ctx* c) {
    if (!c) return IQPT_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    if (c->stream3) (void)hipStreamSynchronize(c->stream3);
    free_comm(c);
    free_scene(c);
    if (c->d_lin) (void)hipFree(c->d_lin);
    if (c->d_bgra_own) (void)hipFree(c->d_bgra_own);
    else if (c->d_bgra) (void)hipFree(c->d_bgra);       // (a context whose creation failed half way)
    if (c->d_alt_own) (void)hipFree(c->d_alt_own);
    for (int i = 0; i < iqpt::kPipeRing; ++i) {
        if (c->d_pring[i]) (void)hipFree(c->d_pring[i]);
        if (c->pev[i]) (void)hipEventDestroy(c->pev[i]);
    }
    if (c->d_rng) (void)hipFree(c->d_rng);
    if (c->d_rays) (void)hipFree(c->d_rays);
    if (c->d_queue) (void)hipFree(c->d_queue);
    for (uint32_t* b : {c->d_tile_done, c->d_xcd_order, c->d_xcd_band, c->d_ovl_err})
        if (b) (void)hipFree(b);
    if (c->ev_pre) (void)hipEventDestroy(c->ev_pre);
    if (c->ev_s2) (void)hipEventDestroy(c->ev_s2);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->stream3) (void)hipStreamDestroy(c->stream3);
    if (c->ev_pipe_end) (void)hipEventDestroy(c->ev_pipe_end);
    free_split(c);
    for (void* b : {(void*)c->d_spec, (void*)c->d_spec_res, (void*)c->d_spec_tl, (void*)c->d_spec_plan,
})
        if (b) (void)hipFree(b);
    for (void* b : {(void*)c->h_spec_rho, (void*)c->h_spec_plan})
        if (b) (void)hipHostFree(b);
    for (hipEvent_t e : {c->ev_spec_rho, c->ev_spec_plan})
        if (e) (void)hipEventDestroy(e);
    if (c->d_stats) (void)hipFree(c->d_stats);
    if (c->d_cull) (void)hipFree(c->d_cull);
    if (c->d_certain) (void)hipFree(c->d_certain);
    if (c->d_sky_tiles) (void)hipFree(c->d_sky_tiles);
    if (c->ev_sky) (void)hipEventDestroy(c->ev_sky);
    if (c->d_tile_order) (void)hipFree(c->d_tile_order);
    if (c->d_list) (void)hipFree(c->d_list);
    if (c->d_pmask) (void)hipFree(c->d_pmask);
    for (auto& tl : c->timed)
        for (hipEvent_t ev : {tl.e0, tl.e1, tl.e1b})
            if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : c->event_pool) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : c->tune_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return IQPT_OK;
}

int iqpt_set_camera(iqpt_ctx* c, const iqpt_camera* cam) {
    if (!c || !cam) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (cam->width != c->width || cam->height != c->height)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "camera size differs from the context frame");
    // an interactive loop sets the camera every frame: the same view keeps its tile masks and the
    // camera-ray path decision (only a changed view is binned and timed again)
    if (c->have_camera && std::memcmp(&c->cam, cam, sizeof *cam) == 0) return IQPT_OK;
    c->cam = *cam;   // passed by value to every launch: no device copy to race with
    c->have_camera = true;
    c->cull_valid = false;
    c->tune_stage = 0;              // the faster camera-ray path depends on the view: time it again
    return IQPT_OK;
}

int iqpt_upload_packet(iqpt_ctx* c, const iqpt_packet_desc* pk) {
    if (!c || !pk) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    const uint32_t ntdc = pk->num_drawcalls[IQPT_MESH_TRIANGLES];
    const uint32_t nsdc = pk->num_drawcalls[IQPT_MESH_SPHERES];
    if ((ntdc && !pk->tri_mesh_dcs) || (nsdc && !pk->sphere_dcs) || (pk->num_tri_meshes && !pk->tri_meshes))
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "packet array is NULL");
    // world-space relayout (the ray-independent part of path_tracer.cu:257-270)
    std::vector<float4_storage> tris, shade, sph;
    uint64_t total = 0;
    for (uint32_t i = 0; i < ntdc; ++i) {
        const uint32_t id = pk->tri_mesh_dcs[i].mesh_id;
        if (id >= pk->num_tri_meshes)
            return iqpt::fail(IQPT_ERR_INVALID_ARG, "tri drawcall " + std::to_string(i) + ": mesh_id out of range");
        const iqpt_tri_mesh& m = pk->tri_meshes[id];
        if (m.num_indices % 3 != 0)
            return iqpt::fail(IQPT_ERR_INVALID_ARG, "mesh " + std::to_string(id) + ": num_indices not a multiple of 3");
        if (m.num_indices && (!m.indices || !m.vertices))
            return iqpt::fail(IQPT_ERR_INVALID_ARG, "mesh " + std::to_string(id) + ": NULL arrays");
        total += m.num_indices / 3;
    }
    if (total > 0xffffffffull / 4) return iqpt::fail(IQPT_ERR_INVALID_ARG, "too many triangles");
    // sphere indices, pair counts ((n + 1) / 2) and mask words are 32-bit in the kernels
    if (nsdc > 0xffffffffu / 4) return iqpt::fail(IQPT_ERR_INVALID_ARG, "too many spheres");
    // material table (iqpt.h): indices in range, known types
    if (pk->materials) {
        if ((ntdc && !pk->tri_dc_material) || (nsdc && !pk->sphere_dc_material))
            return iqpt::fail(IQPT_ERR_INVALID_ARG, "material table without per-drawcall indices");
        for (uint32_t i = 0; i < ntdc; ++i)
            if (pk->tri_dc_material[i] >= pk->num_materials)
                return iqpt::fail(IQPT_ERR_INVALID_ARG, "tri drawcall " + std::to_string(i) + ": material out of range");
        for (uint32_t i = 0; i < nsdc; ++i)
            if (pk->sphere_dc_material[i] >= pk->num_materials)
                return iqpt::fail(IQPT_ERR_INVALID_ARG, "sphere drawcall " + std::to_string(i) + ": material out of range");
        for (uint32_t k = 0; k < pk->num_materials; ++k)
            if (pk->materials[k].type != IQPT_MAT_EMISSIVE && pk->materials[k].type != IQPT_MAT_OREN_NAYAR)
                return iqpt::fail(IQPT_ERR_INVALID_ARG, "material " + std::to_string(k) + ": unknown type");
    }
    tris.reserve(total * iqpt::kTriFloat4);
    shade.reserve(total * 3);
    for (uint32_t i = 0; i < ntdc; ++i) {
        const iqpt_tri_mesh_drawcall& dc = pk->tri_mesh_dcs[i];
        const iq::mat4 M = iq::mat4::from(dc.transform);
        const iq::mat4 N = iq::normal_matrix(M);                     // path_tracer.cu:260
        const iqpt_tri_mesh& m = pk->tri_meshes[dc.mesh_id];
        for (uint32_t j = 0; j < m.num_indices; j += 3) {
            const uint32_t ia = m.indices[j], ib = m.indices[j + 1], ic = m.indices[j + 2];
            if (ia >= m.num_vertices || ib >= m.num_vertices || ic >= m.num_vertices)
                return iqpt::fail(IQPT_ERR_INVALID_ARG, "mesh " + std::to_string(dc.mesh_id) + ": index out of range");
            const iqpt_vertex& a = m.vertices[ia];
            const iqpt_vertex& b = m.vertices[ib];
            const iqpt_vertex& cc = m.vertices[ic];
            const iq::vec4 v0 = iq::transformed(iq::load3(a.pos, iq::usage::POINT), M);
            const iq::vec4 v1 = iq::transformed(iq::load3(b.pos, iq::usage::POINT), M);
            const iq::vec4 v2 = iq::transformed(iq::load3(cc.pos, iq::usage::POINT), M);
            const iq::vec4 n0 = iq::transformed(iq::load3(a.normal, iq::usage::DIRECTION), N);
            const iq::vec4 n1 = iq::transformed(iq::load3(b.normal, iq::usage::DIRECTION), N);
            const iq::vec4 n2 = iq::transformed(iq::load3(cc.normal, iq::usage::DIRECTION), N);
            const iq::vec4 e1 = v1 - v0, e2 = v2 - v0;               // shape.cu:65-66
            const iq::vec4 ng = iq::cross3(e1, e2);                  // shape.cu:98
            tris.push_back({v0.x, v0.y, v0.z, e1.x});
            tris.push_back({e1.y, e1.z, e2.x, e2.y});
            tris.push_back({e2.z, 0.0f, 0.0f, 0.0f});
            shade.push_back({n0.x, n0.y, n0.z, ng.x});
            shade.push_back({n1.x, n1.y, n1.z, ng.y});
            shade.push_back({n2.x, n2.y, n2.z, ng.z});
        }
    }
    for (uint32_t i = 0; i < nsdc; ++i) {
        const iqpt_sphere_drawcall& s = pk->sphere_dcs[i];
        sph.push_back({s.center[0], s.center[1], s.center[2], s.radius});
    }
    // material records: (albedo.rgb, type bits), (strength | sigma, A, B, 0) with the Oren-Nayar
    // constants of material.cu:22-24 evaluated here by the same IEEE operations (sigma clamped to
    // [0, 1] as the oren_nayar constructor does, material.h:25-29)
    std::vector<float4_storage> mats;
    std::vector<uint32_t> tri_mat, sph_mat;
    if (pk->materials) {
        for (uint32_t k = 0; k < pk->num_materials; ++k) {
            const iqpt_material& m = pk->materials[k];
            float tbits;
            std::memcpy(&tbits, &m.type, 4);
            mats.push_back({m.albedo[0], m.albedo[1], m.albedo[2], tbits});
            if (m.type == IQPT_MAT_EMISSIVE) {
                mats.push_back({m.param, 0.0f, 0.0f, 0.0f});
            } else {
                const float sigma = m.param < 0.0f ? 0.0f : (m.param > 1.0f ? 1.0f : m.param);
                const float sigma2 = sigma * sigma;
                const float A = 1.0f - 0.5f * sigma2 / (sigma2 + 0.33f);
                const float B = 0.45f * sigma2 / (sigma2 + 0.09f);
                mats.push_back({sigma, A, B, 0.0f});
            }
        }
        for (uint32_t i = 0; i < ntdc; ++i) {
            const iqpt_tri_mesh& m = pk->tri_meshes[pk->tri_mesh_dcs[i].mesh_id];
            tri_mat.insert(tri_mat.end(), m.num_indices / 3, pk->tri_dc_material[i]);
        }
        sph_mat.assign(pk->sphere_dc_material, pk->sphere_dc_material + nsdc);
    }
    // kOptFastDiv (iq_fastdiv.h): iq_rcp is exact for |x| in [2^-126, 2^126) and for 0, inf, NaN.
    // Möller–Trumbore determinants are |e1 . (dir x e2)| <= |e1| |e2| (|dir| = 1) < 2^126 when every
    // finite edge component is within 2^60 (a non-finite component makes det inf or NaN), and sphere
    // radii must be 0, non-finite or in [2^-126, 2^126).
    bool fast_rcp_ok = true;
    auto big = [](float v) { return std::isfinite(v) && std::fabs(v) > 0x1p60f; };
    for (uint64_t k = 0; k < total && fast_rcp_ok; ++k) {
        const float4_storage* t = &tris[k * iqpt::kTriFloat4];
        fast_rcp_ok = !(big(t[0].w) || big(t[1].x) || big(t[1].y) || big(t[1].z) || big(t[1].w) || big(t[2].x));
    }
    for (const float4_storage& s : sph) {
        const float r = std::fabs(s.w);
        if (std::isfinite(r) && r != 0.0f && (r < 0x1p-126f || r >= 0x1p126f)) fast_rcp_ok = false;
    }
    // pair layouts (iqpt_internal.hpp): SoA inside each pair of consecutive primitives
    std::vector<float4_storage> tri_pairs, sph_pairs;
    const size_t ntp = (total + 1) / 2, nsp = ((size_t)nsdc + 1) / 2;
    tri_pairs.resize(ntp * iqpt::kTriPairFloat4, float4_storage{0.0f, 0.0f, 0.0f, 0.0f});
    for (size_t k = 0; k < total; ++k) {
        const float4_storage* t = &tris[k * iqpt::kTriFloat4];
        const float f[9] = {t[0].x, t[0].y, t[0].z, t[0].w, t[1].x, t[1].y, t[1].z, t[1].w, t[2].x};
        float* dst = &tri_pairs[(k / 2) * iqpt::kTriPairFloat4].x;     // 20 floats, component c at 2c + (k & 1)
        for (int comp = 0; comp < 9; ++comp) dst[2 * comp + (k & 1)] = f[comp];
    }
    sph_pairs.resize(nsp * iqpt::kSphPairFloat4, float4_storage{0.0f, 0.0f, 0.0f, 0.0f});
    for (size_t k = 0; k < nsdc; ++k) {
        const float f[4] = {sph[k].x, sph[k].y, sph[k].z, sph[k].w};
        float* dst = &sph_pairs[(k / 2) * iqpt::kSphPairFloat4].x;
        for (int comp = 0; comp < 4; ++comp) dst[2 * comp + (k & 1)] = f[comp];
    }
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));   // a render in flight may still read the old scene
    free_scene(c);
    c->have_packet = false;
    auto upload = [&](const std::vector<float4_storage>& v, float4_storage** dst) -> int {
        if (v.empty()) return IQPT_OK;
        if (hipMalloc(dst, v.size() * sizeof(float4_storage)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "scene allocation");
        IQPT_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(float4_storage), hipMemcpyHostToDevice));
        return IQPT_OK;
    };
    bvh_host bvh;
    const bool have_bvh = build_bvh(tris, sph, bvh);
    sbvh_host sbvh;
    const bool have_sbvh = build_sbvh(sph, sbvh);
    auto upload_u32 = [&](const std::vector<uint32_t>& v, uint32_t** dst) -> int {
        if (v.empty()) return IQPT_OK;
        if (hipMalloc(dst, v.size() * sizeof(uint32_t)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "material index allocation");
        IQPT_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        return IQPT_OK;
    };
    if ((st = upload(tris, &c->d_tris)) || (st = upload(tri_pairs, &c->d_tri_pairs)) ||
        (st = upload(shade, &c->d_tri_shade)) || (st = upload(sph, &c->d_sph)) ||
        (st = upload(sph_pairs, &c->d_sph_pairs)) || (st = upload(mats, &c->d_mats)) ||
        (st = upload_u32(tri_mat, &c->d_tri_mat)) || (st = upload_u32(sph_mat, &c->d_sph_mat)) ||
        (have_bvh && ((st = upload(bvh.nodes, &c->d_bvh_nodes)) || (st = upload(bvh.pairs, &c->d_bvh_pairs)) ||
                      (st = upload_u32(bvh.always, &c->d_bvh_always)))) ||
        (have_sbvh && ((st = upload(sbvh.nodes, &c->d_sbvh_nodes)) || (st = upload(sbvh.sph, &c->d_sbvh_sph)) ||
                       (st = upload_u32(sbvh.idx, &c->d_sbvh_idx)) ||
                       (st = upload_u32(sbvh.always, &c->d_sbvh_always))))) {
        free_scene(c);
        return st;
    }
    if (have_sbvh) {
        c->sbvh_nnodes = (uint32_t)(sbvh.nodes.size() / iqpt::kSphNodeFloat4);
        c->sbvh_nalways = (uint32_t)sbvh.always.size();
        c->sbvh_gulp = sbvh.gulp;
    }
    if (have_bvh) {
        c->bvh_nnodes = (uint32_t)(bvh.nodes.size() / iqpt::kBvhNodeFloat4);
        c->bvh_nalways = (uint32_t)bvh.always.size();
        c->bvh_md = bvh.md;
        c->bvh_gulp = bvh.gulp;
    }
    c->ntri = (uint32_t)total;
    c->nsph = nsdc;
    c->h_sph = sph;
    c->fast_rcp_ok = fast_rcp_ok;
    c->have_packet = true;
    return IQPT_OK;
}

namespace {
int render_launch(iqpt_ctx* c, uint32_t spp);
}

int iqpt_render(iqpt_ctx* c, uint32_t spp) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (!c->have_camera || !c->have_packet) return iqpt::fail(IQPT_ERR_NOT_READY, "camera and packet must be set");
    if (spp == 0) return IQPT_OK;
    int st = use_device(c);
    if (st) return st;
    // launches of at most kAccTableMax samples, so the running-mean table always covers the launch
    // (a pixel's samples are sequential either way: same bits as one launch)
    while (spp > 0) {
        const uint32_t n = std::min(spp, iqpt::kAccTableMax);
        if ((st = render_launch(c, n)) != IQPT_OK) return st;
        spp -= n;
    }
    return IQPT_OK;
}

namespace {
int render_launch(iqpt_ctx* c, uint32_t spp) {
    int st = IQPT_OK;
    iqpt::kparams p;
    std::memset(&p, 0, sizeof p);
    p.width = c->width;
    p.height = c->height;
    p.x0 = c->set.x0;
    p.ncols = c->ncols;
    p.y0 = c->set.y0;
    p.ystep = c->set.ystep;
    p.nrows = c->set.nrows;
    p.npix = c->npix;
    p.frame0 = c->frame;
    p.spp = spp;
    p.max_depth = c->max_depth;
    std::memcpy(p.inv_proj, c->cam.inv_proj, sizeof p.inv_proj);
    std::memcpy(p.inv_view, c->cam.inv_view, sizeof p.inv_view);
    cam_constants(c->cam, &p.cam_const, &p.cam_near_rw, &p.cam_far_rw);
    p.acc_tab = spp <= iqpt::kAccTableMax ? 1u : 0u;
    p.spin_limit = c->spin_limit;
    p.iter_limit = c->iter_limit;
    p.frames32 = (c->frame + (uint64_t)spp) < (1ull << 32) ? 1u : 0u;
    // running mean under kOptFastDiv: c / n by Markstein's correction is exact while the quotient is
    // normal, c >= 2^-125 n; with n <= frame0 + spp the threshold 2^-124 (frame0 + spp) (rounded up,
    // at least 2^-100 for the operand range) routes the rest to the IEEE division (mean_terms)
    {
        const double nmax = (double)(c->frame + (uint64_t)spp);
        p.mean_tiny = (float)std::max(std::ldexp(nmax, -124) * 2.0, std::ldexp(1.0, -99));
    }
    p.tris = c->d_tris;
    p.tri_pairs = c->d_tri_pairs;
    p.ntri = c->ntri;
    p.ntri_pairs = (c->ntri + 1) / 2;
    p.spheres = c->d_sph;
    p.sph_pairs = c->d_sph_pairs;
    p.nsph = c->nsph;
    p.nsph_pairs = (c->nsph + 1) / 2;
    // kOptFastDiv only for packets inside its range (upload) and frames up to 2^24 wide / high
    // (camera_ray divides by W and H with the pre-rounded reciprocals below)
    int opt = c->opt;
    if (!c->fast_rcp_ok || c->width > (1u << 24) || c->height > (1u << 24)) opt &= ~iqpt::kOptFastDiv;
    if (!(opt & iqpt::kOptPair)) opt &= ~iqpt::kOptCull;       // masks are per primitive pair
    if (c->d_mats) opt |= iqpt::kOptMaterials;                  // the packet carries a material table
    p.tri_mat = c->d_tri_mat;
    p.sph_mat = c->d_sph_mat;
    if (c->d_bvh_nodes && c->bvh_nnodes) {
        p.bvh_nodes = c->d_bvh_nodes;
        p.bvh_pairs = c->d_bvh_pairs;
        p.bvh_always = c->d_bvh_always;
        p.bvh_nnodes = c->bvh_nnodes;
        p.bvh_nalways = c->bvh_nalways;
        p.bvh_md = c->bvh_md;
        p.bvh_gulp = c->bvh_gulp;
    }
    if (c->d_sbvh_nodes && c->sbvh_nnodes) {
        p.sbvh_nodes = c->d_sbvh_nodes;
        p.sbvh_sph = c->d_sbvh_sph;
        p.sbvh_idx = c->d_sbvh_idx;
        p.sbvh_always = c->d_sbvh_always;
        p.sbvh_nnodes = c->sbvh_nnodes;
        p.sbvh_nalways = c->sbvh_nalways;
        p.sbvh_gulp = c->sbvh_gulp;
        p.bvh_md = 1.001f;          // bvh_ray_ok: |d_i| bound shared with the triangle BVH
    }
    p.mats = c->d_mats;
    p.tri_shade = c->d_tri_shade;
    // no sphere, no material table: every triangle emissive, a ray decided by its first accepted triangle
    p.anyhit = (c->nsph == 0 && !c->d_mats && c->anyhit_on) ? 1u : 0u;
    p.rcp_width = 1.0f / (float)c->width;
    p.rcp_height = 1.0f / (float)c->height;
    const bool cam_axis = (opt & iqpt::kOptCamConst) && cam_axis_constants(c->cam, p.cam_ax);
    const bool pair = (opt & iqpt::kOptPair) != 0;
    const uint32_t tri_rec = pair ? iqpt::kTriPairFloat4 * 16 : iqpt::kTriFloat4 * 16;   // bytes per LDS record
    const uint32_t sph_rec = pair ? iqpt::kSphPairFloat4 * 16 : 16;
    const uint32_t tri_recs = pair ? p.ntri_pairs : p.ntri;
    const uint32_t sph_recs = pair ? p.nsph_pairs : p.nsph;
    const uint64_t resident = (uint64_t)tri_recs * tri_rec + (uint64_t)sph_recs * sph_rec;
    const bool stream_batches = resident > iqpt::kLdsResidentBytes;
    // production streamed variants are built without the 5-wave bound (registers for the BVH)
    if (stream_batches && !iqpt::render_variant_exists(c->max_depth, true, opt) &&
        iqpt::render_variant_exists(c->max_depth, true, opt & ~iqpt::kOptLB5))
        opt &= ~iqpt::kOptLB5;
    // streamed any-hit scenes take the variants with the first-hit exits (kOptAnyHit), where one exists
    if (stream_batches && p.anyhit && iqpt::render_variant_exists(c->max_depth, true, opt | iqpt::kOptAnyHit))
        opt |= iqpt::kOptAnyHit;
    // kOptCamAxis: the short camera transform, kept only where the camera qualifies (a caller's option
    // mask may ask for it; production launches add it below, where a variant exists: DESIGN.md §3.8)
    if (!cam_axis) opt &= ~iqpt::kOptCamAxis;
    // resident production variants carry kOptPrio (VALU priority for scatter-heavy waves; same bits)
    if (!stream_batches && !iqpt::render_variant_exists(c->max_depth, false, opt) &&
        iqpt::render_variant_exists(c->max_depth, false, opt | iqpt::kOptPrio))
        opt |= iqpt::kOptPrio;
    if (stream_batches) {
        p.tri_batch = pair ? iqpt::kTriBatch / 2 : iqpt::kTriBatch;   // records
        p.sph_batch = pair ? iqpt::kSphBatch / 2 : iqpt::kSphBatch;
        // a wave takes new pixels once this many of its lanes are idle (64: a whole tile at a time, its rays
        // coherent through the BVHs)
        p.refill_min = std::min<uint32_t>(64u, std::max<uint32_t>(1u, c->stream_refill_min));
    } else {
        p.refill_min = std::min<uint32_t>(64u, std::max<uint32_t>(1u, c->resident_refill_min));
        p.tri_batch = tri_recs;
        p.sph_batch = sph_recs;
    }
    // scene batch + running-mean table (padded to 16 B) + (kOptCull) one uint4 slot per thread +
    // the scatter-record stack (max_depth - 1 records per thread; one float each)
    uint32_t lds = p.tri_batch * tri_rec + p.sph_batch * sph_rec +
                         (p.acc_tab ? ((spp + 1u) & ~1u) * 8u + ((spp + 3u) & ~3u) * 4u : 0u) +
                         ((opt & iqpt::kOptCull) ? iqpt::kRenderBlock * 16u : 0u) +
                         (uint32_t)std::max(c->max_depth, 1) * iqpt::kRenderBlock * 4u *
                             ((opt & iqpt::kOptMaterials) ? 3u : 1u);
    if ((opt & iqpt::kOptCull) && (c->ntri + c->nsph) > 0) {
        if (!c->cull_valid) {
            if ((st = join_streams(c)) != IQPT_OK) return st;   // new masks and tile lists: the chain restarts
            if ((st = build_cull(c)) != IQPT_OK) return st;
        }
        p.cull = c->d_cull;
        p.certain = c->certain_valid && c->certain_on ? c->d_certain : nullptr;
        p.tile_order = c->d_tile_order;
        p.cull_ntx = c->cull_ntx;
        p.cull_wt = c->cull_wt;
        p.cull_stride = c->cull_stride;
        if (c->d_list) {
            p.list = c->d_list;
            p.list_off_tri = c->d_list + c->list_total;
            p.list_off_sph = p.list_off_tri + (c->cull_ntx * c->cull_nty + 1);
            if (c->d_pmask) {
                const uint32_t nt = c->cull_ntx * c->cull_nty;
                p.pmask_off = c->d_pmask;
                p.pmask = c->d_pmask + (nt + 1);
                p.pmask_certain = c->d_pmask + (nt + 1) + c->pmask_words;
            }
        }
    }
    p.ntx = (c->ncols + iqpt::kCullTile - 1) / iqpt::kCullTile;
    p.ntiles = p.ntx * ((c->set.nrows + iqpt::kCullTile - 1) / iqpt::kCullTile);
    p.lin = c->d_lin;
    p.bgra = c->d_bgra;
    p.rng = c->d_rng;
    p.rays = c->d_rays;
    p.queue = c->d_queue;
    p.stats = c->d_stats;
    // any-hit scenes whose every tile list has per-pixel masks: iqpt_anyhit_kernel renders the launch (one camera
    // ray per sample, the lane's own candidates; no BVH-primary tuning, no queue)
    const bool anyk = c->pmask_mode == 2 && !c->opt_fixed && stream_batches && p.anyhit && (opt & iqpt::kOptAnyHit) &&
                      p.pmask != nullptr && c->pmask_all && p.list != nullptr && spp > 0 && spp <= iqpt::kAccTableMax &&
                      iqpt::anyhit_variant_exists(opt);
    // kOptBvhPrimary: decided by timing (see iqpt_ctx::tune_stage). Its batch-free variants keep the 5-wave bound
    // the batched streamed variants drop for launches of up to kPrimaryLB5MaxSpp samples, and run at 4 waves
    // per SIMD (no spills) above that where that variant is built: C5 16 spp 54.0-54.3 -> 51.5 ms, 1 spp 3.17 ->
    // 3.39 ms (r06 run 36)
    constexpr uint32_t kPrimaryLB5MaxSpp = 4;
    const bool prim_lb5 = spp <= kPrimaryLB5MaxSpp ||
                          !iqpt::render_variant_exists(c->max_depth, true, (opt | iqpt::kOptBvhPrimary) & ~iqpt::kOptLB5);
    const int prim_opt = ((opt | iqpt::kOptBvhPrimary) & ~iqpt::kOptLB5) |
                         (prim_lb5 && iqpt::render_variant_exists(c->max_depth, true,
                                                                  opt | iqpt::kOptBvhPrimary | iqpt::kOptLB5)
                              ? iqpt::kOptLB5 : 0);
    int tune_slot = -1;
    if (!c->opt_fixed && !anyk && stream_batches && p.bvh_nodes && p.cull && (opt & iqpt::kOptBvh) &&
        iqpt::render_variant_exists(c->max_depth, true, prim_opt)) {
        if (c->tune_stage == iqpt::kTuneLaunches) {
            // per variant the fastest of its timed launches, per sample-pixel of work
            double best[2] = {1e300, 1e300};
            bool ok = hipEventSynchronize(c->tune_ev[2 * iqpt::kTuneLaunches - 1]) == hipSuccess;
            for (int s = 0; ok && s < iqpt::kTuneLaunches; ++s) {
                float ms = 0.0f;
                ok = hipEventElapsedTime(&ms, c->tune_ev[2 * s], c->tune_ev[2 * s + 1]) == hipSuccess;
                if (ok) best[s & 1] = std::min(best[s & 1], (double)ms / std::max(1.0, c->tune_work[s]));
            }
            c->tune_primary = ok && best[1] < best[0];
            c->tune_stage = iqpt::kTuneLaunches + 1;
        }
        if (c->tune_stage < iqpt::kTuneLaunches) {
            tune_slot = c->tune_stage;
            for (int k = 0; k < 2; ++k) {
                hipEvent_t& ev = c->tune_ev[2 * tune_slot + k];
                if (!ev && hipEventCreate(&ev) != hipSuccess) ev = nullptr;
                if (!ev) tune_slot = -1;
            }
            if (tune_slot == 0) {   // load both code objects before either is timed
                int o2 = 0;
                (void)iqpt::render_occupancy(c->max_depth, true, prim_opt, lds, &o2);
            }
        }
        if ((tune_slot >= 0 && (tune_slot & 1)) || (tune_slot < 0 && c->tune_primary)) opt = prim_opt;
    }
    // kOptSplit: resident scenes with a split set, when the mode asks for it (auto:
    // fewer owned pixels than kSplitAutoPixelsPerLane per resident lane, i.e. too few pixel chains to
    // fill and drain the chip evenly)
    // (round 6: the chain kernel, DESIGN.md §3.9, and FAN launches, §3.10, left the library for the branch
    // round6-ab-archive; AUTO never chose FAN, and chain launches only where spec launches did not fit)
    bool auto_spec = false;             // AUTO: the share is small enough for spec launches (if they apply)
    if (c->split_mode == IQPT_SPLIT_AUTO && !stream_batches && p.cull && c->n_split_tiles > 0 && tune_slot < 0 &&
        !(opt & iqpt::kOptMaterials) && spp <= iqpt::kAccTableMax) {
        int occ_p = 0;
        if (iqpt::render_occupancy(c->max_depth, false, opt, lds, &occ_p) != 0) occ_p = 0;
        const double lanes = (double)c->num_cus * std::max(occ_p, 1) * iqpt::kRenderBlock;
        auto_spec = (double)c->npix < iqpt::kSpecAutoPixelsPerLane * lanes;
    }
    // the fan kernel: the anchored tiles (no sphere candidate) of spec and split launches
    const bool fan_ok = !stream_batches && p.cull && (c->n_anchor > 0 || c->n_fan_tiles > 0) && tune_slot < 0 &&
                        !(opt & iqpt::kOptMaterials) && spp <= iqpt::kAccTableMax && c->cull_wt <= 16 &&
                        iqpt::fan_variant_exists(opt);
    // spec launches: sphere pixels slot-parallel, every other pixel in the fan kernel
    bool spec = fan_ok && (c->split_mode == IQPT_SPLIT_SPEC || auto_spec) && c->n_split_tiles > 0 &&
                iqpt::spec_variant_exists(c->max_depth, opt) &&
                (size_t)c->n_chain_pix * ((iqpt::kSplitMCapMul * spp + 15u) & ~15u) * 16u <= iqpt::kSplitResBudget;
    if (spec) {
        // the block's LDS (scene, tables, slot marks: 32 pixels x the window cap) must fit the device's per-block
        // limit with at least one resident block, else the plain path (same bits; ADVICE r3: a 1,024-spp launch
        // with a scene near the resident limit needs ~170 KB)
        iqpt::kspec probe;
        std::memset(&probe, 0, sizeof probe);
        probe.m_cap = (iqpt::kSplitMCapMul * spp + 15u) & ~15u;
        int occ_s = 0;
        spec = iqpt::spec_lds(p, probe) <= c->lds_per_block && probe.m_cap <= 65535u &&
               iqpt::spec_occupancy(p, probe, opt, &occ_s) == 0 && occ_s >= 1;
        (void)hipGetLastError();
    }
    uint32_t lds_split = lds + iqpt::kRenderBlock * (16u + 24u);   // + lds_sp and the base states
    bool split = false;
    if (!spec && c->split_mode != IQPT_SPLIT_OFF && c->split_mode != IQPT_SPLIT_SPEC && !stream_batches && p.cull &&
        c->n_split_tiles > 0 &&
        tune_slot < 0 && iqpt::render_variant_exists(c->max_depth, false, opt | iqpt::kOptSplit)) {
        int occ_s = 0;
        if (iqpt::render_occupancy(c->max_depth, false, opt | iqpt::kOptSplit, lds_split, &occ_s) != 0) occ_s = 0;
        const double lanes = (double)c->num_cus * std::max(occ_s, 1) * iqpt::kRenderBlock;
        split = occ_s > 0 && (c->split_mode == IQPT_SPLIT_ON || (double)c->npix < iqpt::kSplitAutoPixelsPerLane * lanes);
    }
    // pipelined spec launches continue without a join (the launch below orders itself); the others never overlap
    const bool pipe_next = c->pipe && spec && c->specfan_mode == 0 && c->pipe_kind == 1;
    if ((split || spec) && !pipe_next && (st = join_streams(c)) != IQPT_OK) return st;
    // split launches with the anchored tiles in the fan kernel beside the four split passes
    const bool fan_split = split && fan_ok;
    const size_t ns_cap = (size_t)c->n_split_tiles * iqpt::kQueueChunk;
    const uint32_t m_cap = (iqpt::kSplitMCapMul * spp + 15u) & ~15u;
    const uint32_t g_max = (m_cap + iqpt::kSplitRunLen - 1) / iqpt::kSplitRunLen;
    if (split && (size_t)m_cap * ns_cap > c->res_slots) {
        if (c->d_res || c->d_nres || c->d_run_st || c->d_chunks) {
            IQPT_HIP(hipStreamSynchronize(c->stream));
            for (void* b : {(void*)c->d_res, (void*)c->d_nres, (void*)c->d_run_st, (void*)c->d_chunks})
                if (b) (void)hipFree(b);
            c->d_res = nullptr;
            c->d_nres = nullptr;
            c->d_run_st = nullptr;
            c->d_chunks = nullptr;
            c->res_slots = 0;
        }
        const size_t slots = (size_t)m_cap * ns_cap;
        const size_t st_words = (size_t)(g_max + 1) * 6 * ns_cap;
        const size_t chunk_words = 2 * (size_t)g_max * c->n_split_tiles;
        if (slots * (sizeof(float4_storage) + 1) + (st_words + chunk_words) * 4 <= iqpt::kSplitResBudget &&
            hipMalloc(&c->d_res, slots * sizeof(float4_storage)) == hipSuccess &&
            hipMalloc(&c->d_nres, slots) == hipSuccess &&
            hipMalloc(&c->d_run_st, st_words * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc(&c->d_chunks, chunk_words * sizeof(uint32_t)) == hipSuccess) {
            c->res_slots = slots;
        } else {
            (void)hipGetLastError();
            split = false;     // over the budget: the plain kernel (same bits)
        }
    }
    iqpt::ksplit ks;
    std::memset(&ks, 0, sizeof ks);
    if (split) {
        opt |= iqpt::kOptSplit;
        lds = lds_split;
        uint32_t* base = c->d_split;
        uint32_t* sp_pix = base + c->n_anchor + c->n_split_tiles;
        p.anchor_order = base;
        p.n_anchor = c->n_anchor;
        p.n_split_tiles = c->n_split_tiles;
        p.split_tiles = base + c->n_anchor;
        p.chunks = c->d_chunks;
        p.chunk_count = c->d_queue + 3;
        p.split_len = iqpt::kSplitRunLen;
        p.run_st = c->d_run_st;
        p.refill_min = std::min<uint32_t>(64u, std::max<uint32_t>(1u, c->split_refill_min));
        p.ns_cap = (uint32_t)ns_cap;
        p.m_cap = m_cap;
        p.sp_pix = sp_pix;
        p.sp_win = sp_pix + ns_cap;
        p.sp_rho = sp_pix + 2 * ns_cap;
        p.left = sp_pix + 3 * ns_cap;
        p.left_count = c->d_queue + 2;
        p.res = c->d_res;
        p.nres = c->d_nres;
        p.sp_st = c->d_sp_st;
        p.sp_acc = c->d_sp_acc;
        ks.ns_cap = (uint32_t)ns_cap;
        ks.spp = spp;
        ks.m_cap = m_cap;
        ks.g_max = g_max;
        ks.run_len = iqpt::kSplitRunLen;
        ks.heavy_rho = c->split_heavy_rho;
        ks.run_st = c->d_run_st;
        ks.split_tiles = base + c->n_anchor;
        ks.chunks = c->d_chunks;
        ks.chunk_count = c->d_queue + 3;
        ks.max_depth = c->max_depth;
        ks.frame0 = c->frame;
        ks.mean_tiny = p.mean_tiny;
        ks.npix = c->npix;
        ks.ncols = c->ncols;
        ks.nrows = c->set.nrows;
        ks.sp_pix = sp_pix;
        ks.sp_win = sp_pix + ns_cap;
        ks.sp_rho = sp_pix + 2 * ns_cap;
        ks.left = sp_pix + 3 * ns_cap;
        ks.left_count = c->d_queue + 2;
        ks.res = c->d_res;
        ks.nres = c->d_nres;
        ks.sp_st = c->d_sp_st;
        ks.sp_acc = c->d_sp_acc;
        ks.lin = c->d_lin;
        ks.bgra = c->d_bgra;
        ks.rng = c->d_rng;
        ks.rays = c->d_rays;
        if (!c->split_last) {
            // no chain history from the previous launch (new split set or the plain kernel ran)
            IQPT_HIP(hipMemsetAsync(sp_pix + 2 * ns_cap, 0, ns_cap * sizeof(uint32_t), c->stream));
        }
    }
    // kOptOverlap: resident, culled, not split, not a tuning launch
    // Tiles are bound to the 8 XCDs (HW_REG_XCC_ID): only on a device that exposes 8 (not a partition
    // mode) and with at least 64 blocks, so that the observed round-robin dispatch puts blocks on every
    // XCD (HIP promises no placement; the kernel's last block checks it and raises an error bit if not)
    // kOptPipe: plain launches over resident scenes under the reference's materials take the
    // two-rays-per-lane variants where they are built (a caller's fixed option set keeps its own bits)
    if (!c->opt_fixed && c->pipe_on && !stream_batches && !split && !spec && tune_slot < 0 &&
        p.cull != nullptr && p.acc_tab && !(opt & iqpt::kOptMaterials) &&
        iqpt::render_variant_exists(c->max_depth, false, opt | iqpt::kOptPipe))
        opt |= iqpt::kOptPipe;
    bool ovl = c->overlap_mode != IQPT_OVERLAP_OFF && !stream_batches && !split && !spec &&
               p.cull != nullptr &&
               tune_slot < 0 && c->d_tile_done && c->d_xcd_order && c->num_xcc == 8 && c->num_cus >= 64 &&
               (uint64_t)c->npix >= 64ull * iqpt::kRenderBlock &&
               iqpt::render_variant_exists(c->max_depth, false, opt | iqpt::kOptOverlap);
    int occ = 0;
    if (iqpt::render_occupancy(c->max_depth, stream_batches, ovl ? (opt | iqpt::kOptOverlap) : opt, lds, &occ) != 0 ||
        occ < 1)
        occ = 1;
    // two launches in flight: each keeps one block slot per CU free for the other (occ - 1 per CU), so the
    // earlier launch, which the later one waits for, can always run
    if (ovl && occ < 2) ovl = false;
    if ((ovl || fan_split || spec) && !c->stream2) {
        if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_pre, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_s2, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            if (fan_split || spec) return iqpt::fail(IQPT_ERR_HIP, "second stream for the spec / fan kernel");
            ovl = false;
            c->overlap_mode = IQPT_OVERLAP_OFF;
        }
    }
    if (!ovl && !pipe_next && (st = join_streams(c)) != IQPT_OK) return st;
    hipStream_t ls = c->stream;                       // the launch's stream
    if (ovl) {
        opt |= iqpt::kOptOverlap;
        if (c->ovl_zero || c->ovl_epoch >= (1u << 24)) {
            if ((st = join_streams(c)) != IQPT_OK) return st;
            IQPT_HIP(hipMemsetAsync(c->d_tile_done, 0, (size_t)p.ntiles * sizeof(uint32_t), c->stream));
            c->ovl_zero = false;
            c->ovl_epoch = 0;
        }
        if (!c->next_on_main) {
            // after everything `stream` held before its last launch, that launch's list resets included
            ls = c->stream2;
            IQPT_HIP(hipStreamWaitEvent(c->stream2, c->ev_pre, 0));
            c->s2_pending = true;
        }
        const uint32_t parity = c->ovl_epoch & 1u;
        p.queue = c->d_queue + 4 + parity * (iqpt::kOverlapQueueWords / 2);
        p.tile_done = c->d_tile_done;
        p.done_target = c->ovl_epoch ? c->ovl_epoch + c->wait_bias : 0u;
        p.xcd_order = c->d_xcd_order;
        std::memcpy(p.xcd_off, c->xcd_off, sizeof p.xcd_off);
        p.ovl_err = c->d_ovl_err;
        if (c->copy_seq > c->pwaited) {    // copies behind earlier pipelined launches may still read d_bgra
            IQPT_HIP(hipStreamWaitEvent(ls, c->pev[c->copy_seq % iqpt::kPipeRing], 0));
            c->pwaited = c->copy_seq;
        }
        if (c->d_bgra_alt) {
            std::swap(c->d_bgra, c->d_bgra_alt);
            p.bgra = c->d_bgra;
        }
        IQPT_HIP(hipMemsetAsync(p.queue, 0, (iqpt::kOverlapQueueWords / 2) * sizeof(uint32_t), ls));
        // the next launch (stream2) starts after all of this but not after this launch
        if (ls == c->stream) IQPT_HIP(hipEventRecord(c->ev_pre, c->stream));
        occ -= 1;
    }
    // pitch-only cameras take the short camera transform (exact, kOptCamAxis) wherever that variant is
    // built: resident plain, overlapped and spec launches (C2 -14 % overlapped, C3 shares -3..-12 %,
    // profiles/r02/ab_camaxis_overlap.json, split_share_v17_camaxis.json)
    if (!c->opt_fixed && cam_axis && !stream_batches && !split &&
        iqpt::render_variant_exists(c->max_depth, false, opt | iqpt::kOptCamAxis) &&
        (!spec || iqpt::spec_variant_exists(c->max_depth, opt | iqpt::kOptCamAxis)))
        opt |= iqpt::kOptCamAxis;
    const uint64_t want = ((uint64_t)c->npix + iqpt::kRenderBlock - 1) / iqpt::kRenderBlock;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->num_cus * occ));
    // streamed scenes: per-XCD tile lists and queue words (iqpt_debug_set_stream_xcd), where the overlapped
    // launches could bind tiles to XCDs (8 XCDs, enough blocks; the kernel's last block checks the placement)
    constexpr uint32_t kStreamXcdMaxSpp = 4;
    const int xmode = c->stream_xcd == 3 ? (spp <= kStreamXcdMaxSpp ? 1 : 0) : c->stream_xcd;
    const bool xcdq = stream_batches && xmode != 0 && p.cull && c->d_xcd_order && c->d_xcd_band &&
                      !split && !spec && c->num_xcc == 8 && c->num_cus >= 64 && grid >= 64;
    if (xcdq) {
        p.xcd_order = xmode == 1 ? c->d_xcd_order : c->d_xcd_band;
        std::memcpy(p.xcd_off, xmode == 1 ? c->xcd_off : c->xcd_band_off, sizeof p.xcd_off);
        p.ovl_err = c->d_ovl_err;
    }
    if (!ovl && !spec)
        IQPT_HIP(hipMemsetAsync(c->d_queue, 0, (xcdq ? 16u * 8u + 1u : 4u) * sizeof(uint32_t), c->stream));
    hipEvent_t e0 = take_event(c), e1 = take_event(c), e1b = nullptr;
    // pipelined spec launches: the timing events are recorded by the spec and fan kernels' dispatches (no
    // marker packets between consecutive kernels on the two streams: -0.012 ms per step at N = 8, -0.04 with
    // a copy and gather every step, r04 run 12)
    const bool bind_spec = spec && c->specfan_mode == 0 && c->n_chain_pix > 0;
    // overlapped launches: recorded by the launch's first kernel on `ls` (the sky kernel or the plain kernel)
    // and its last (the plain kernel)
    const bool bind_ovl = ovl && tune_slot < 0;
    bool e0_bound = false, e1_bound = false;
    if (e0 && !bind_spec && !bind_ovl) (void)hipEventRecord(e0, ls);
    if (tune_slot >= 0) (void)hipEventRecord(c->tune_ev[2 * tune_slot], c->stream);
    int le = 0;
    // pipelined launches (spec, FAN): the frame buffer this launch writes (the other one once copies are
    // asynchronous), after the copy that read it two launches ago; the second stream after everything
    // `stream` held unless the launch continues a pipeline
    auto pipe_begin = [&]() -> int {
        if (c->pring_on) {
            c->pidx = (c->pidx + 1) % iqpt::kPipeRing;
            c->d_bgra = c->d_pring[c->pidx];
            p.bgra = c->d_bgra;
            if (c->pseq[c->pidx] > c->pwaited) {
                const uint64_t tgt = std::max<uint64_t>(c->pseq[c->pidx], c->copy_seq > 2u ? c->copy_seq - 2u : 0u);
                if (!(c->gather_skip & 4)) {
                    IQPT_HIP(hipStreamWaitEvent(c->stream, c->pev[tgt % iqpt::kPipeRing], 0));
                    IQPT_HIP(hipStreamWaitEvent(c->stream2, c->pev[tgt % iqpt::kPipeRing], 0));
                }
                c->pwaited = tgt;
            }
        }
        if (!pipe_next) {
            IQPT_HIP(hipEventRecord(c->ev_pre, c->stream));
            IQPT_HIP(hipStreamWaitEvent(c->stream2, c->ev_pre, 0));
        }
        return IQPT_OK;
    };
    // ... and its end: no join; the copy stream and every other entry point wait for both streams
    auto pipe_end = [&](int kind) -> int {
        if (!c->ev_pipe_end && hipEventCreateWithFlags(&c->ev_pipe_end, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            return iqpt::fail(IQPT_ERR_HIP, "pipelined launch events");
        }
        if (int s = ensure_copy_stream(c)) return s;
        // the kernels' own end events (bound timing events) where there are some; otherwise a copy records
        // markers on both streams when it is asked for
        c->end1 = e1_bound ? e1 : nullptr;
        c->end2 = e1b;
        if (!e1b) {
            e1b = take_event(c);
            if (e1b) (void)hipEventRecord(e1b, c->stream2);
        }
        c->s2_pending = true;
        c->pipe = le == 0;
        c->pipe_kind = kind;
        return IQPT_OK;
    };
    // ---- the spec kernel's buffers, parameters, plan and history (pipelined spec launches on `stream`):
    // every enqueue of these on the spec kernel's stream `ss`
    auto spec_buffers = [&](hipStream_t ss, iqpt::kspec& ks2) -> int {
        std::memset(&ks2, 0, sizeof ks2);
        const uint32_t n = c->n_chain_pix;
        const uint32_t m_cap = (iqpt::kSplitMCapMul * spp + 15u) & ~15u;
        if (n > 0 && n <= c->spec_n && m_cap > c->spec_mcap) {
            // a longer launch on the same pixel list: only the slot results grow (the history and the plan stay)
            IQPT_HIP(hipStreamSynchronize(c->stream));
            if (c->d_spec_res) (void)hipFree(c->d_spec_res);
            c->d_spec_res = nullptr;
            c->spec_mcap = 0;
            const size_t slots = (size_t)c->spec_n * m_cap;
            if (slots * 16 > iqpt::kSplitResBudget ||
                hipMalloc(&c->d_spec_res, slots * sizeof(float4_storage)) != hipSuccess) {
                (void)hipGetLastError();
                c->d_spec_res = nullptr;
                return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "spec slot results");
            }
            c->spec_mcap = m_cap;
        }
        if (n > 0 && n > c->spec_n) {
            IQPT_HIP(hipStreamSynchronize(c->stream));
            for (void* b : {(void*)c->d_spec, (void*)c->d_spec_res, (void*)c->d_spec_plan})
                if (b) (void)hipFree(b);
            for (void* b : {(void*)c->h_spec_rho, (void*)c->h_spec_plan})
                if (b) (void)hipHostFree(b);
            c->d_spec = nullptr;
            c->d_spec_res = nullptr;
            c->d_spec_plan = nullptr;
            c->h_spec_rho = c->h_spec_plan = nullptr;
            c->spec_n = c->spec_mcap = 0;
            c->spec_plan_n = 0;
            c->spec_rho_pending = c->spec_plan_up = false;
            const size_t slots = (size_t)n * m_cap;
            if ((!c->ev_spec_rho && hipEventCreateWithFlags(&c->ev_spec_rho, hipEventDisableTiming) != hipSuccess) ||
                (!c->ev_spec_plan && hipEventCreateWithFlags(&c->ev_spec_plan, hipEventDisableTiming) != hipSuccess) ||
                slots * 16 > iqpt::kSplitResBudget ||
                hipMalloc(&c->d_spec, (2 * (size_t)n + 2) * sizeof(uint32_t)) != hipSuccess ||
                hipMalloc(&c->d_spec_res, slots * sizeof(float4_storage)) != hipSuccess ||
                hipMalloc(&c->d_spec_plan, 3 * (size_t)n * sizeof(uint32_t)) != hipSuccess ||
                hipHostMalloc(&c->h_spec_rho, (size_t)n * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc(&c->h_spec_plan, 3 * (size_t)n * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "spec buffers");
            }
            // the statistics counters run from here (iqpt_debug_spec_info reads and clears them)
            IQPT_HIP(hipMemsetAsync(c->d_spec + 2 * (size_t)n, 0, 2 * sizeof(uint32_t), ss));
            c->spec_n = n;
            c->spec_mcap = m_cap;
            c->spec_rho_valid = false;
        }
        p.ovl_err = c->d_ovl_err;
        ks2.n = n;
        ks2.m_cap = m_cap;
        ks2.rho0 = c->spec_rho0;
        ks2.margin_div = c->spec_margin_div;
        ks2.parity_rho = c->spec_parity_rho;
        ks2.parity_hi = c->spec_parity_hi;
        ks2.pix = c->d_chain_pix;
        ks2.m = c->d_spec;
        ks2.rho = c->d_spec + n;
        ks2.run_count = c->d_spec + 2 * (size_t)n;
        ks2.res = c->d_spec_res;
        // a new pixel list: no history, and the statistics counters behind it (d_spec + 2 n) restart too
        // (after a list that shrank n they pointed into the old history)
        if (n > 0 && !c->spec_rho_valid) IQPT_HIP(hipMemsetAsync(ks2.rho, 0, ((size_t)n + 2) * sizeof(uint32_t), ss));
        c->spec_rho_valid = c->spec_rho_valid || n > 0;
        return IQPT_OK;
    };
    auto spec_plan = [&](hipStream_t ss, iqpt::kspec& ks2) -> int {
        const uint32_t n = ks2.n;
        // the plan: built from the history read after an earlier launch (asynchronous), or, for tests,
        // synchronously from the current history
        if (n > 0 && c->spec_plan_mode >= 2) {
            IQPT_HIP(hipStreamSynchronize(ss));
            IQPT_HIP(hipMemcpy(c->h_spec_rho, ks2.rho, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
            const uint32_t nb = spec_build_plan(c, p, ks2, opt, c->h_spec_rho, c->h_spec_plan);
            IQPT_HIP(hipMemcpy(c->d_spec_plan, c->h_spec_plan, ((size_t)n + 2 * (size_t)nb) * sizeof(uint32_t),
                               hipMemcpyHostToDevice));
            c->spec_plan_n = n;
            c->spec_plan_blocks = nb;
        } else if (n > 0 && c->spec_plan_mode == 1 && c->spec_rho_pending &&
                   hipEventQuery(c->ev_spec_rho) == hipSuccess &&
                   (!c->spec_plan_up || hipEventQuery(c->ev_spec_plan) == hipSuccess)) {
            const uint32_t nb = spec_build_plan(c, p, ks2, opt, c->h_spec_rho, c->h_spec_plan);
            IQPT_HIP(hipMemcpyAsync(c->d_spec_plan, c->h_spec_plan, ((size_t)n + 2 * (size_t)nb) * sizeof(uint32_t),
                                    hipMemcpyHostToDevice, ss));
            IQPT_HIP(hipEventRecord(c->ev_spec_plan, ss));
            c->spec_plan_up = true;
            c->spec_rho_pending = false;
            c->spec_plan_n = n;
            c->spec_plan_blocks = nb;
            c->spec_plan_age = 0;
        }
        if (n > 0 && c->spec_plan_mode >= 1 && c->spec_plan_n == n) {
            ks2.order = c->d_spec_plan;
            ks2.blocks = c->d_spec_plan + n;
            ks2.nblocks = c->spec_plan_blocks;
        }
        if (c->spec_tl_on && n > 0) {
            const size_t nb = ks2.blocks ? ks2.nblocks : (n + iqpt::kSpecPixPerBlock - 1) / iqpt::kSpecPixPerBlock;
            if (nb > c->spec_tl_blocks) {
                IQPT_HIP(hipStreamSynchronize(ss));
                if (c->d_spec_tl) (void)hipFree(c->d_spec_tl);
                c->d_spec_tl = nullptr;
                c->spec_tl_blocks = 0;
                if (hipMalloc(&c->d_spec_tl, nb * 8 * sizeof(unsigned long long)) != hipSuccess) {
                    (void)hipGetLastError();
                    return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "spec timeline");
                }
                c->spec_tl_blocks = nb;
            }
            IQPT_HIP(hipMemsetAsync(c->d_spec_tl, 0, nb * 8 * sizeof(unsigned long long), ss));
            ks2.tl = c->d_spec_tl;
        }
        return IQPT_OK;
    };
    // read this launch's history for the next plan: before the first plan, then every kSpecReplan launches
    auto spec_history = [&](hipStream_t ss, const iqpt::kspec& ks2) -> int {
        const uint32_t n = ks2.n;
        if (n > 0 && c->spec_plan_mode == 1 && !c->spec_rho_pending &&
            (c->spec_plan_n != n || ++c->spec_plan_age >= iqpt::kSpecReplan)) {
            IQPT_HIP(hipMemcpyAsync(c->h_spec_rho, ks2.rho, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, ss));
            IQPT_HIP(hipEventRecord(c->ev_spec_rho, ss));
            c->spec_rho_pending = true;
        }
        return IQPT_OK;
    };
    // certain-miss pixels: plain launches hand them to iqpt_sky_kernel, ahead of the plain
    // kernel on the launch's stream; the plain kernel skips them. Consecutive sky kernels order themselves
    // through ev_sky (overlapped launches alternate streams); their pixels are disjoint from the plain kernel's.
    const bool sky = c->sky_on && c->certain_on && c->certain_valid && c->n_sky_tiles > 0 && p.certain != nullptr &&
                     !stream_batches && !split && !spec && tune_slot < 0 &&
                     !(opt & iqpt::kOptMaterials) && spp <= iqpt::kAccTableMax && iqpt::sky_variant_exists(opt);
    // overlapped launches may put the sky kernel behind the plain kernel on the launch's stream
    // (iqpt_debug_set_sky_order), so the plain kernel, whose sphere tiles carry the launch's longest chains,
    // is not queued behind it
    const bool sky_deferred = sky && ovl && bind_ovl && c->sky_after;
    if (sky) {
        p.miss = c->d_certain + 2 * (size_t)c->cull_ntx * c->cull_nty;
        if (!c->ev_sky && hipEventCreateWithFlags(&c->ev_sky, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            return iqpt::fail(IQPT_ERR_HIP, "sky kernel event");
        }
        if (!sky_deferred) {
            const hipStream_t ss = ovl ? ls : c->stream;
            if (c->sky_last && c->sky_last != ss) IQPT_HIP(hipStreamWaitEvent(ss, c->ev_sky, 0));
            const bool b0 = bind_ovl && e0 && p.spp > 0;
            if (b0) iqpt::bind_launch_events(e0, nullptr);
            le = iqpt::launch_sky(ss, p, c->d_sky_tiles, c->n_sky_tiles, opt);
            iqpt::bind_launch_events(nullptr, nullptr);
            e0_bound = b0 && le == 0;
            if (le != 0) return iqpt::hip_fail((hipError_t)le, "sky kernel launch");
            IQPT_HIP(hipEventRecord(c->ev_sky, ss));
            c->sky_last = ss;
        }
    }
    if (ovl) {
        if (bind_ovl) iqpt::bind_launch_events(e0_bound ? nullptr : e0, sky_deferred ? nullptr : e1);
        le = iqpt::launch_render(ls, p, grid, lds, stream_batches, opt);
        iqpt::bind_launch_events(nullptr, nullptr);
        if (bind_ovl) {
            if (le != 0 && e0 && !e0_bound) (void)hipEventRecord(e0, ls);   // (not read: the launch failed)
            e0_bound = true;
            e1_bound = le == 0 && e1 != nullptr && !sky_deferred;
        }
        if (sky_deferred && le == 0) {
            if (c->sky_last && c->sky_last != ls) IQPT_HIP(hipStreamWaitEvent(ls, c->ev_sky, 0));
            iqpt::bind_launch_events(nullptr, e1);
            le = iqpt::launch_sky(ls, p, c->d_sky_tiles, c->n_sky_tiles, opt);
            iqpt::bind_launch_events(nullptr, nullptr);
            e1_bound = le == 0 && e1 != nullptr;
            if (le != 0) return iqpt::hip_fail((hipError_t)le, "sky kernel launch");
            IQPT_HIP(hipEventRecord(c->ev_sky, ls));
            c->sky_last = ls;
        }
        c->ovl_epoch += 1;
        c->next_on_main = !c->next_on_main;
        if (le != 0) c->ovl_zero = true;     // a failed launch breaks the chain's counts: restart it
    } else if (spec) {
        // every pixel without a sphere in reach in the fan kernel on stream2; the sphere pixels in
        // iqpt_spec_kernel on stream (slots, then the walk)
        iqpt::kspec ks2;
        if ((st = spec_buffers(c->stream, ks2)) != IQPT_OK) return st;
        if (c->specfan_mode == 0 && (st = pipe_begin()) != IQPT_OK) return st;
        iqpt::kparams pf = p;
        pf.tile_order = c->d_fan_tiles;
        pf.fan_lanes = c->d_fan_lanes;
        // the certain-miss pixels the fan lists left out: the sky kernel, ahead of the fan
        // kernel on its stream (consecutive launches' sky kernels are ordered there)
        if (c->sky_active) {
            iqpt::kparams pm = pf;
            pm.miss = c->d_certain + 2 * (size_t)c->cull_ntx * c->cull_nty;
            le = iqpt::launch_sky(c->specfan_mode == 0 ? c->stream2 : c->stream, pm, c->d_sky_tiles, c->n_sky_tiles, opt);
            if (le != 0) return iqpt::hip_fail((hipError_t)le, "sky kernel launch");
        }
        if ((st = spec_plan(c->stream, ks2)) != IQPT_OK) return st;
        const uint32_t n = ks2.n;
        auto run_spec = [&]() -> int { return iqpt::launch_spec(c->stream, p, ks2, opt); };
        if (c->specfan_mode == 1) {
            if (n > 0) le = run_spec();
            if (le == 0 && c->n_fan_tiles > 0) le = iqpt::launch_fan(c->stream, pf, c->n_fan_tiles, opt);
        } else {
            if (n > 0) {
                iqpt::bind_launch_events(e0, e1);
                le = run_spec();
                iqpt::bind_launch_events(nullptr, nullptr);
                e1_bound = le == 0 && e1 != nullptr;
                if (le != 0 && e0) (void)hipEventRecord(e0, c->stream);   // (unrecorded events are not read)
            }
            if (le == 0 && c->n_fan_tiles > 0) {
                e1b = take_event(c);
                iqpt::bind_launch_events(nullptr, e1b);
                le = iqpt::launch_fan(c->stream2, pf, c->n_fan_tiles, opt);
                iqpt::bind_launch_events(nullptr, nullptr);
                if (le != 0 && e1b) {
                    c->event_pool.push_back(e1b);
                    e1b = nullptr;
                }
            }
            if ((st = pipe_end(1)) != IQPT_OK) return st;
        }
        if (le == 0 && (st = spec_history(c->stream, ks2)) != IQPT_OK) return st;
    } else if (split) {
        // prep -> round 1 (runs, anchored tiles, light split pixels) -> stitch -> round 2 (leftovers); with
        // the fan kernel the anchored tiles leave round 1 for iqpt_fan_kernel on stream2
        if (fan_split) {
            iqpt::kparams pf = p;
            pf.tile_order = c->d_split;
            IQPT_HIP(hipEventRecord(c->ev_pre, c->stream));
            IQPT_HIP(hipStreamWaitEvent(c->stream2, c->ev_pre, 0));
            le = iqpt::launch_fan(c->stream2, pf, c->n_anchor, opt);
            p.n_anchor = 0;
        }
        if (le == 0) le = iqpt::launch_split_prep(c->stream, ks);
        p.split_round = 1;
        p.queue = c->d_queue;
        if (le == 0) le = iqpt::launch_render(c->stream, p, grid, lds, stream_batches, opt);
        if (le == 0) le = iqpt::launch_split_stitch(c->stream, ks, (opt & iqpt::kOptFastDiv) != 0);
        p.split_round = 2;
        p.queue = c->d_queue + 1;
        if (le == 0) le = iqpt::launch_render(c->stream, p, grid, lds, stream_batches, opt);
        if (fan_split) {
            IQPT_HIP(hipEventRecord(c->ev_s2, c->stream2));
            IQPT_HIP(hipStreamWaitEvent(c->stream, c->ev_s2, 0));
        }
    } else if (anyk) {
        le = iqpt::launch_anyhit(c->stream, p, opt);
    } else {
        le = iqpt::launch_render(c->stream, p, grid, lds, stream_batches, opt);
    }
    c->last_anyk = anyk;
    c->split_last = split;
    c->fan_last = fan_split || spec;
    c->spec_last = spec;
    c->last_ls = ls;
    c->last_ovl = ovl;
    c->last_xcd_lists = (ovl || xcdq) && !spec && !split && !anyk;
    if (tune_slot >= 0) (void)hipEventRecord(c->tune_ev[2 * tune_slot + 1], c->stream);
    if (e1 && !e1_bound) (void)hipEventRecord(e1, ls);
    if (e0 && e1) c->timed.push_back({e0, e1, e1b});
    if (le != 0) return iqpt::hip_fail((hipError_t)le, "render kernel launch");
    c->last_opt = opt;
    if (tune_slot >= 0) {
        c->tune_work[tune_slot] = (double)spp * (double)c->npix;
        c->tune_stage = tune_slot + 1;
    }
    c->frame += spp;
    return IQPT_OK;
}
}  // namespace

int iqpt_sync(iqpt_ctx* c) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    // a per-tile wait that gave up or a chain wave past its bound (never expected) leaves the frame
    // undefined: report it (and keep reporting it, iqpt_ctx::dev_err)
    return check_dev_err(c);
}

int iqpt_reset(iqpt_ctx* c) {                                       // path_tracer.cu:394-400
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    IQPT_HIP(hipMemsetAsync(c->d_bgra, 0, (size_t)c->npix * sizeof(uint32_t), c->stream));
    IQPT_HIP(hipStreamSynchronize(c->stream));
    c->frame = 0;
    return IQPT_OK;
}

int iqpt_read(iqpt_ctx* c, float* lin_rgba, uint8_t* bgra) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    if (lin_rgba && (st = fetch_compact(c, c->d_lin, 4, 1, lin_rgba)) != IQPT_OK) return st;
    // the BGRA8 frame is stored in compact order already (tile_to_compact)
    if (bgra) IQPT_HIP(hipMemcpyAsync(bgra, c->d_bgra, (size_t)c->npix * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                      c->stream));
    IQPT_HIP(hipStreamSynchronize(c->stream));
    return check_dev_err(c);
}

int iqpt_read_rng(iqpt_ctx* c, uint32_t* states) {
    if (!c || !states) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    std::vector<uint32_t> planes((size_t)c->npix * 6);
    if ((st = fetch_compact(c, c->d_rng, 1, 6, planes.data())) != IQPT_OK) return st;
    if ((st = check_dev_err(c)) != IQPT_OK) return st;
    for (size_t p = 0; p < c->npix; ++p)
        for (int k = 0; k < 6; ++k) states[p * 6 + k] = planes[(size_t)k * c->npix + p];
    return IQPT_OK;
}

int iqpt_copy_accum_device(iqpt_ctx* c, void* dst_device, size_t bytes) {
    if (!c || !dst_device) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (bytes < (size_t)c->npix * sizeof(float4_storage)) return iqpt::fail(IQPT_ERR_INVALID_ARG, "destination too small");
    int st = enter(c);
    if (st) return st;
    const int le = iqpt::launch_relayout(c->stream, reinterpret_cast<const uint32_t*>(c->d_lin),
                                         static_cast<uint32_t*>(dst_device), c->ncols, c->set.nrows, 4, 1, true);
    if (le != 0) return iqpt::hip_fail((hipError_t)le, "accumulator reorder");
    IQPT_HIP(hipStreamSynchronize(c->stream));
    return check_dev_err(c);
}

namespace {
// Checkpoint file: header, then accumulator (npix float4), BGRA (npix u32), RNG (6 planes of npix u32).
struct ckpt_header {
    char magic[8];            // "IQPTCKP1"
    uint32_t version;         // 1
    uint32_t width, height;
    uint32_t x0, x1, y0, ystep, nrows;
    int32_t max_depth;
    uint64_t seed;
    uint64_t frame;
    uint64_t rays;
    uint64_t npix;
    uint64_t checksum;        // FNV-1a 64 over the payload
};
constexpr char kCkptMagic[8] = {'I', 'Q', 'P', 'T', 'C', 'K', 'P', '1'};

uint64_t fnv1a(const void* data, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(data);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}
}  // namespace

int iqpt_checkpoint_save(iqpt_ctx* c, const char* path) {
    if (!c || !path) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    const size_t n = c->npix;
    std::vector<float4_storage> lin(n);
    std::vector<uint32_t> bgra(n), rng(n * 6);
    unsigned long long rays = 0;
    // the file holds the compact row-major order (independent of the device layout)
    if ((st = check_dev_err(c)) != IQPT_OK) return st;     // never persist undefined state
    if ((st = fetch_compact(c, c->d_lin, 4, 1, lin.data())) != IQPT_OK ||
        (st = fetch_compact(c, c->d_rng, 1, 6, rng.data())) != IQPT_OK)
        return st;
    IQPT_HIP(hipMemcpy(bgra.data(), c->d_bgra, n * sizeof(uint32_t), hipMemcpyDeviceToHost));   // compact already
    if ((st = read_rays(c, &rays)) != IQPT_OK) return st;
    ckpt_header h;
    std::memset(&h, 0, sizeof h);
    std::memcpy(h.magic, kCkptMagic, 8);
    h.version = 1;
    h.width = c->width;
    h.height = c->height;
    h.x0 = c->set.x0;
    h.x1 = c->set.x1;
    h.y0 = c->set.y0;
    h.ystep = c->set.ystep;
    h.nrows = c->set.nrows;
    h.max_depth = c->max_depth;
    h.seed = c->seed;
    h.frame = c->frame;
    h.rays = rays;
    h.npix = n;
    uint64_t sum = fnv1a(lin.data(), n * sizeof(float4_storage));
    sum = fnv1a(bgra.data(), n * sizeof(uint32_t), sum);
    h.checksum = fnv1a(rng.data(), n * 6 * sizeof(uint32_t), sum);
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return iqpt::fail(IQPT_ERR_INVALID_ARG, "cannot open " + tmp);
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 &&
              std::fwrite(lin.data(), sizeof(float4_storage), n, f) == n &&
              std::fwrite(bgra.data(), sizeof(uint32_t), n, f) == n &&
              std::fwrite(rng.data(), sizeof(uint32_t), n * 6, f) == n * 6;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        return iqpt::fail(IQPT_ERR_INVALID_ARG, std::string("cannot write ") + path);
    }
    return IQPT_OK;
}

int iqpt_checkpoint_load(iqpt_ctx* c, const char* path) {
    if (!c || !path) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) return iqpt::fail(IQPT_ERR_INVALID_ARG, std::string("cannot open ") + path);
    ckpt_header h;
    const size_t n = c->npix;
    std::vector<float4_storage> lin(n);
    std::vector<uint32_t> bgra(n), rng(n * 6);
    bool ok = std::fread(&h, sizeof h, 1, f) == 1;
    std::string why;
    if (!ok || std::memcmp(h.magic, kCkptMagic, 8) != 0 || h.version != 1) why = "not an iqpt checkpoint (v1)";
    else if (h.width != c->width || h.height != c->height || h.x0 != c->set.x0 || h.x1 != c->set.x1 ||
             h.y0 != c->set.y0 || h.ystep != c->set.ystep || h.nrows != c->set.nrows || h.npix != n)
        why = "frame size / pixel set differ from the context";
    else if (h.seed != c->seed || h.max_depth != c->max_depth) why = "seed / max_depth differ from the context";
    if (why.empty()) {
        ok = std::fread(lin.data(), sizeof(float4_storage), n, f) == n &&
             std::fread(bgra.data(), sizeof(uint32_t), n, f) == n &&
             std::fread(rng.data(), sizeof(uint32_t), n * 6, f) == n * 6;
        unsigned char extra;
        if (!ok || std::fread(&extra, 1, 1, f) != 0) why = "truncated or oversized checkpoint";
    }
    std::fclose(f);
    if (why.empty()) {
        uint64_t sum = fnv1a(lin.data(), n * sizeof(float4_storage));
        sum = fnv1a(bgra.data(), n * sizeof(uint32_t), sum);
        if (fnv1a(rng.data(), n * 6 * sizeof(uint32_t), sum) != h.checksum) why = "checksum mismatch";
    }
    // the accumulator's w is 0 from iqpt_create on and the kernel stores it as 0 (a whole float4 per
    // pixel): a checkpoint with another w did not come from a context
    if (why.empty())
        for (size_t i = 0; i < n; ++i)
            if (lin[i].w != 0.0f || std::signbit(lin[i].w)) {
                why = "accumulator w is not +0 (the kernel never produces another)";
                break;
            }
    if (!why.empty()) return iqpt::fail(IQPT_ERR_INVALID_ARG, std::string(path) + ": " + why);
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    const unsigned long long rays = h.rays;
    if ((st = store_compact(c, lin.data(), 4, 1, c->d_lin)) != IQPT_OK ||
        (st = store_compact(c, rng.data(), 1, 6, c->d_rng)) != IQPT_OK)
        return st;
    IQPT_HIP(hipMemcpy(c->d_bgra, bgra.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));   // compact order
    {
        std::vector<unsigned long long> slots((size_t)iqpt::kRaySlots * iqpt::kRaySlotStride, 0ull);
        slots[0] = rays;
        IQPT_HIP(hipMemcpy(c->d_rays, slots.data(), slots.size() * sizeof(unsigned long long), hipMemcpyHostToDevice));
    }
    c->frame = h.frame;
    // the whole pixel state is replaced: a latched kernel error no longer applies
    IQPT_HIP(hipMemset(c->d_ovl_err, 0, sizeof(uint32_t)));
    c->dev_err = 0;
    return IQPT_OK;
}

int iqpt_num_pixels(const iqpt_ctx* c, uint64_t* npix) {
    if (!c || !npix) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *npix = c->npix;
    return IQPT_OK;
}

int iqpt_frame_count(const iqpt_ctx* c, uint64_t* frames) {
    if (!c || !frames) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *frames = c->frame;
    return IQPT_OK;
}

int iqpt_rays_traced(iqpt_ctx* c, uint64_t* rays) {
    if (!c || !rays) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    unsigned long long v = 0;
    if ((st = read_rays(c, &v)) != IQPT_OK) return st;
    *rays = v;
    return IQPT_OK;
}

int iqpt_kernel_time(iqpt_ctx* c, double* total_ms, uint64_t* launches) {
    if (!c || !total_ms || !launches) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    c->end1 = c->end2 = nullptr;        // (the events go back to the pool)
    double sum = 0.0, span = 0.0;
    for (auto& tl : c->timed) {
        float ms = 0.0f, end = 0.0f;
        IQPT_HIP(hipEventElapsedTime(&ms, tl.e0, tl.e1));
        // span: from the first launch's start to the latest end (launches on two streams overlap)
        IQPT_HIP(hipEventElapsedTime(&end, c->timed.front().e0, tl.e1));
        if (tl.e1b) {
            float ms2 = 0.0f, end2 = 0.0f;
            IQPT_HIP(hipEventElapsedTime(&ms2, tl.e0, tl.e1b));
            IQPT_HIP(hipEventElapsedTime(&end2, c->timed.front().e0, tl.e1b));
            ms = std::max(ms, ms2);
            end = std::max(end, end2);
            c->event_pool.push_back(tl.e1b);
        }
        sum += ms;
        span = std::max(span, (double)end);
        c->event_pool.push_back(tl.e0);
        c->event_pool.push_back(tl.e1);
    }
    c->last_span_ms = span;
    *total_ms = sum;
    *launches = c->timed.size();
    c->timed.clear();
    return IQPT_OK;
}

/* Internal (tools): the per-pixel split of the last camera / packet — sphere pixels (the chain and spec
 * kernels' list), fan tiles, anchored tiles, split tiles — and, after a spec launch, the sum of its
 * windows and of its chains' slots per sample, and since the last call (the call clears them) the chains
 * finished past their window (out8[7] low 32 bits) and the parity chains that needed the fix-up pass (out8[7]
 * high 32 bits). Synchronises. */
int iqpt_debug_spec_info(iqpt_ctx* c, unsigned long long* out8) {
    if (!c || !out8) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    for (int i = 0; i < 8; ++i) out8[i] = 0;
    out8[0] = c->n_chain_pix;
    out8[1] = c->n_fan_tiles;
    out8[2] = c->n_anchor;
    out8[3] = c->n_split_tiles;
    if (c->spec_last && c->d_spec && c->spec_n >= c->n_chain_pix) {
        const uint32_t n = c->n_chain_pix;
        std::vector<uint32_t> v(2 * (size_t)n + 2);
        IQPT_HIP(hipMemcpy(v.data(), c->d_spec, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        out8[4] = c->spec_plan_n == n && c->spec_plan_mode ? c->spec_plan_blocks : 0;   // plan blocks (0: none)
        out8[7] = (unsigned long long)v[2 * (size_t)n + 1] | ((unsigned long long)v[2 * (size_t)n] << 32);
        unsigned long long m = 0, rho = 0;
        for (uint32_t q = 0; q < n; ++q) {
            m += v[q];
            rho += v[n + q];
        }
        out8[5] = m;
        out8[6] = rho;
        IQPT_HIP(hipMemset(c->d_spec + 2 * (size_t)n, 0, 2 * sizeof(uint32_t)));
    }
    return IQPT_OK;
}

/* Internal (measurement): record per spec block s_memrealtime stamps (100 MHz) in later spec launches —
 * start, after round 0's slots, after round 0's walk, end | rounds << 48, then the slot-loop iterations of
 * its four waves (8 words per block) — and read the last launch's. */
int iqpt_debug_spec_timeline(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    c->spec_tl_on = on != 0;
    return IQPT_OK;
}

int iqpt_debug_read_spec_timeline(iqpt_ctx* c, unsigned long long* out, uint32_t cap_blocks, uint32_t* n) {
    if (!c || !out || !n) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *n = 0;
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    if (!c->d_spec_tl || !c->spec_last) return IQPT_OK;
    const size_t nspec = c->spec_plan_n == c->n_chain_pix && c->spec_plan_n && c->spec_plan_mode
                             ? c->spec_plan_blocks
                             : (c->n_chain_pix + iqpt::kSpecPixPerBlock - 1) / iqpt::kSpecPixPerBlock;
    const size_t nb = std::min<size_t>(nspec, std::min<size_t>(cap_blocks, c->spec_tl_blocks));
    if (nb) IQPT_HIP(hipMemcpy(out, c->d_spec_tl, nb * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    *n = (uint32_t)nb;
    return IQPT_OK;
}

/* Internal (measurement): the spec plan in use and the history behind it — order (n words), blocks (2 words
 * each, *nb of them) and the sphere pixels' slots per sample x 256 (n words); *n = sphere pixels (0: no plan).
 * Synchronises. */
int iqpt_debug_read_spec_plan(iqpt_ctx* c, uint32_t* order, uint32_t* blocks, uint32_t* rho, uint32_t cap,
                              uint32_t* n, uint32_t* nb) {
    if (!c || !order || !blocks || !rho || !n || !nb) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *n = *nb = 0;
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    const uint32_t np = c->n_chain_pix;
    if (!c->spec_plan_n || c->spec_plan_n != np || np > cap || !c->d_spec_plan) return IQPT_OK;
    IQPT_HIP(hipMemcpy(order, c->d_spec_plan, (size_t)np * sizeof(uint32_t), hipMemcpyDeviceToHost));
    IQPT_HIP(hipMemcpy(blocks, c->d_spec_plan + np, 2 * (size_t)c->spec_plan_blocks * sizeof(uint32_t),
                       hipMemcpyDeviceToHost));
    IQPT_HIP(hipMemcpy(rho, c->d_spec + np, (size_t)np * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *n = np;
    *nb = c->spec_plan_blocks;
    return IQPT_OK;
}

/* Internal (tests, A/B): the spec plan — 0 none (16 lanes per pixel, list order), 1 from an asynchronous
 * read of the history (the default), 2 rebuilt synchronously before every launch, 3 / 4 the same with
 * every pixel on 32 / 64 lanes, 5 the same with the lane count cycling over 8, 16, 24, 32, 48, 64. Drops the plan. */
int iqpt_debug_spec_plan(iqpt_ctx* c, int mode) {
    if (!c || mode < 0 || mode > 5) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL or mode not 0..5");
    c->spec_plan_mode = mode;
    c->spec_plan_n = 0;
    return IQPT_OK;
}

/* Internal (A/B, tests): certain tiles (kparams::certain) folded at once (1, the default) or rendered like
 * every other tile (0). Rebuilds the masks at the next launch. */
int iqpt_debug_set_certain(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    c->certain_on = on != 0;
    c->cull_valid = false;
    return IQPT_OK;
}

/* Internal (A/B, tests): certain-miss pixels rendered by iqpt_sky_kernel beside plain launches (1, the default)
 * or traced by the plain kernel like every other pixel (0). Rebuilds the masks at the next launch. */
int iqpt_debug_set_sky(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    c->sky_on = on != 0;
    c->cull_valid = false;
    return IQPT_OK;
}

/* Internal (A/B): the gather's footprint beside the render kernels, for the next iqpt_comm_init — RCCL's
 * blocks per collective (ncclConfig_t::maxCTAs; 0: RCCL's own choice) and the communicator stream's priority
 * (-1 the lowest; 0 HIP's default, the default; 1 the highest); skip (measurement only, wrong frames): 1 leaves
 * out the collective, 2 the root's assembly, 4 the render streams' waits for the copies of their frame buffers. */
int iqpt_debug_set_gather(iqpt_ctx* c, int ctas, int prio, int skip) {
    if (!c || ctas < 0 || ctas > 64 || prio < -1 || prio > 1 || skip < 0 || skip > 7)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL, ctas not 0..64, prio not -1..1 or skip not 0..7");
    c->gather_ctas = ctas;
    c->gather_prio = prio;
    c->gather_skip = skip;
    return IQPT_OK;
}

/* Internal (A/B): overlapped launches run the sky kernel ahead of the plain kernel on the launch's stream (0)
 * or behind it (1, the default). Same bits either way. */
int iqpt_debug_set_sky_order(iqpt_ctx* c, int after) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    c->sky_after = after != 0;
    return IQPT_OK;
}

/* Internal (A/B): the timing events around launches and gathers (iqpt_kernel_time, iqpt_comm_time) — 1 on (the
 * default), 0 off: those then report nothing. Each event is a packet on its stream between two kernels. */
int iqpt_debug_set_timing(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    c->timing_on = on != 0;
    return IQPT_OK;
}

/* Internal (tools): the certain-miss pixels of the current masks and the tiles holding them. */
int iqpt_debug_sky_info(iqpt_ctx* c, uint32_t* pixels, uint32_t* tiles) {
    if (!c || !pixels || !tiles) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *pixels = c->certain_valid ? c->n_sky_pixels : 0u;
    *tiles = c->certain_valid ? c->n_sky_tiles : 0u;
    return IQPT_OK;
}

/* Internal (tools, tests): certain pixels of the current masks (*n; 0 without masks or flags), the tile
 * count and the tile grid's width in tiles (*ntx) and, if masks is not NULL, up to cap tiles' 64-bit
 * masks (two words per tile). Synchronises. */
int iqpt_debug_certain_tiles(iqpt_ctx* c, uint32_t* n, uint32_t* ntiles, uint32_t* ntx, uint32_t* masks, uint32_t cap) {
    if (!c || !n || !ntiles || !ntx) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *ntx = c->cull_ntx;
    *n = *ntiles = 0;
    int st = enter(c);
    if (st) return st;
    if (!c->certain_valid || !c->d_certain) return IQPT_OK;
    const uint32_t nt = c->cull_ntx * c->cull_nty;
    std::vector<uint32_t> v(2 * (size_t)nt);
    IQPT_HIP(hipMemcpy(v.data(), c->d_certain, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < v.size(); ++i) *n += (uint32_t)__builtin_popcount(v[i]);
    *ntiles = nt;
    if (masks) std::memcpy(masks, v.data(), std::min<size_t>(v.size(), 2 * (size_t)cap) * sizeof(uint32_t));
    return IQPT_OK;
}

/* Internal (tests, A/B): any-hit queries for triangle-only scenes under the reference's materials (1, the
 * default) or the closest-hit search (0). Same bits either way. */
int iqpt_debug_set_anyhit(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    c->anyhit_on = on != 0;
    c->cull_valid = false;               // the candidate lists' order follows the setting
    return IQPT_OK;
}

/* Internal (tests, A/B): per-pixel candidate masks over the streamed kernel's tile lists: 2 (the default) with
 * iqpt_anyhit_kernel for any-hit scenes whose every tile has them, 1 in the plain kernel only, 0 none (the whole
 * list for every lane). Same bits either way. */
int iqpt_debug_set_pixel_masks(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    if (on < 0 || on > 2) return iqpt::fail(IQPT_ERR_INVALID_ARG, "pixel mask mode must be 0, 1 or 2");
    c->pmask_mode = on;
    c->cull_valid = false;
    return IQPT_OK;
}

/* Internal (tests, tools): tiles whose triangle lists have per-pixel masks (0: none built), whether every tile has
 * them and no tile has a sphere candidate (iqpt_anyhit_kernel's condition besides an any-hit scene), and the longest
 * triangle list (null: not wanted). */
int iqpt_debug_pixel_mask_info(iqpt_ctx* c, uint32_t* tiles, int* all, uint32_t* list_max) {
    if (!c || !tiles || !all) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *tiles = c->pmask_tiles;
    *all = c->pmask_all ? 1 : 0;
    if (list_max) *list_max = c->list_max;
    return IQPT_OK;
}

/* Internal (tests, A/B): resident plain launches under the reference's materials trace the lane's path ray and
 * its pixel's next camera ray together (kOptPipe, 1, the default) or one ray per iteration (0). Same bits either
 * way. */
int iqpt_debug_set_two_ray(iqpt_ctx* c, int on) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    c->pipe_on = on != 0;
    return IQPT_OK;
}

/* Internal (tests, A/B): idle lanes a wave of a streamed-scene launch waits for before it takes new pixels
 * (1..64; 1 = every iteration with an idle lane, round 4; 64, a whole tile at a time, by default). Same bits
 * either way. */
int iqpt_debug_set_stream_refill(iqpt_ctx* c, uint32_t lanes) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (lanes < 1u || lanes > 64u) return iqpt::fail(IQPT_ERR_INVALID_ARG, "lanes 1..64");
    c->stream_refill_min = lanes;
    return IQPT_OK;
}

/* Internal (tests, A/B): how streamed-scene launches deal tiles — 0 one queue over the cost order, 1 per-XCD
 * queues over the cost order dealt round-robin, 2 per-XCD queues over bands of tile rows dealt round-robin
 * (spatially coherent work per XCD L2), 3 (default) 1 for launches of up to 4 samples per pixel, else 0. Same
 * bits either way. */
int iqpt_debug_set_stream_xcd(iqpt_ctx* c, int mode) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (mode < 0 || mode > 3) return iqpt::fail(IQPT_ERR_INVALID_ARG, "mode 0..3");
    c->stream_xcd = mode;
    return IQPT_OK;
}

/* Internal (tests, A/B): the same for the plain kernel's launches over resident scenes (1 by default; split
 * launches keep their own, iqpt_debug_set_split_knobs). Same bits either way. */
int iqpt_debug_set_resident_refill(iqpt_ctx* c, uint32_t lanes) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (lanes < 1u || lanes > 64u) return iqpt::fail(IQPT_ERR_INVALID_ARG, "lanes 1..64");
    c->resident_refill_min = lanes;
    return IQPT_OK;
}

/* Internal (tests, A/B): the spec kernel's parity pixels — a pixel whose last chain took at least rho256 / 256
 * slots per sample traces the even slots of its window first and the odd ones only from where its chain lands on
 * one (pooled over the block's lanes); 0 traces every slot of every window (round 4). Same bits either way. */
int iqpt_debug_set_spec_parity(iqpt_ctx* c, uint32_t rho256) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    c->spec_parity_rho = rho256;
    return IQPT_OK;
}

/* Internal (A/B, measurement): how spec launches run the fan tiles beside the sphere pixels — 0 two kernels on
 * two streams, pipelined across launches (the default), 1 two kernels one after the other on one stream. (Round
 * 4's mode 2, spec and fan blocks in one grid, measured slower and is archived: branch round4-ab-archive.)
 * `lead` is ignored. */
int iqpt_debug_set_specfan(iqpt_ctx* c, int mode, uint32_t lead) {
    (void)lead;
    if (!c || mode < 0 || mode > 1) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL or mode not 0..1");
    int st = enter(c);
    if (st) return st;
    c->specfan_mode = mode;
    return IQPT_OK;
}

/* Internal (tests, A/B): the slots per sample (x 256) a spec window assumes for a pixel without history (a
 * small value makes the chains of sphere pixels leave their first window: the walker then finishes them)
 * and the window margin divisor. 0 restores a default; the history is dropped. */
int iqpt_debug_set_spec(iqpt_ctx* c, uint32_t rho0, uint32_t margin_div) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    c->spec_margin_div = margin_div ? margin_div : 16u;
    c->spec_rho0 = rho0 ? rho0 : iqpt::kSpecRho0;
    c->spec_rho_valid = false;
    return IQPT_OK;
}

/* Internal (tests): after joining the context's streams, fills the LDS of every CU with non-zero garbage (blocks of
 * the largest per-block allocation, eight per CU) on the context's stream, ahead of the next launch, which then
 * starts joined behind it: a kernel that reads LDS before writing it gives other bits than the oracle. */
int iqpt_debug_poison_lds(iqpt_ctx* c, uint32_t pattern) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    int st = enter(c);
    if (st) return st;
    const uint32_t bytes = c->lds_per_block & ~3u;
    const int le = iqpt::launch_lds_poison(c->stream, pattern, bytes, (uint32_t)c->num_cus * 8u);
    if (le != 0) return iqpt::hip_fail((hipError_t)le, "LDS poison kernel");
    IQPT_HIP(hipStreamSynchronize(c->stream));
    return IQPT_OK;
}

/* Internal (tests): lower the kernels' forward-progress bound (0 keeps the default) and bias the per-tile wait targets
 * of overlapped launches, so that tests can force the error path. iter_limit bounded the archived chain kernel's loop
 * (kept in the signature, unused). */
int iqpt_debug_set_limits(iqpt_ctx* c, uint32_t spin_limit, uint32_t iter_limit, uint32_t wait_bias) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    c->spin_limit = spin_limit ? spin_limit : iqpt::kOverlapSpinLimit;
    c->iter_limit = iter_limit ? iter_limit : iqpt::kChainIterLimit;
    c->wait_bias = wait_bias;
    return IQPT_OK;
}

/* Internal (tools/ab_kernel.py): select the kernel option mask of a context and read the
 * diagnostic counters of kOptStats variants. Not part of include/iqpt.h. */
int iqpt_copy_frame_device(iqpt_ctx* c, void* dst_device, size_t bytes) {
    if (!c || !dst_device) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (bytes < (size_t)c->npix * sizeof(uint32_t)) return iqpt::fail(IQPT_ERR_INVALID_ARG, "destination too small");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipMemcpyAsync(dst_device, c->d_bgra, (size_t)c->npix * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                            c->stream));                    // compact order already
    IQPT_HIP(hipStreamSynchronize(c->stream));
    return check_dev_err(c);
}

namespace {
// The stream-ordered frame copy (iqpt_copy_frame_device_async, the gather's send copy): the BGRA8 frame in
// compact order into dst, behind every render issued so far; `wait` (if not null) is waited for on the copy's
// stream first; *used = that stream.
// Pipelined launches, from the first copy or gather behind one on: the ring of frame buffers the launches write
// in turn (each of frame_words(c): the multi-GPU gather sends a launch's buffer as it is).
int ensure_ring(iqpt_ctx* c) {
    if (c->pring_on) return IQPT_OK;
    for (int i = 0; i < iqpt::kPipeRing; ++i) {
        if ((!c->d_pring[i] && hipMalloc(&c->d_pring[i], frame_words(c) * sizeof(uint32_t)) != hipSuccess) ||
            (!c->pev[i] && hipEventCreateWithFlags(&c->pev[i], hipEventDisableTiming) != hipSuccess)) {
            (void)hipGetLastError();
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "frame buffers for pipelined copies");
        }
        c->pseq[i] = 0;
    }
    c->pidx = iqpt::kPipeRing - 1;     // the next launch writes d_pring[0]
    c->pring_on = true;
    return IQPT_OK;
}

int copy_frame_async(iqpt_ctx* c, uint32_t* dst, hipEvent_t wait, hipStream_t* used) {
    // no synchronisation here: an error the kernels raise for this launch is reported by the next
    // synchronising call (iqpt_sync, iqpt_read, ...); one already latched fails the copy now
    if (c->dev_err) return check_dev_err(c);
    int st = IQPT_OK;
    hipStream_t cs = c->stream;
    if (c->pipe) {
        // pipelined spec launches: the copy on stream3 behind both kernels of the last launch; from here on
        // the launches write the ring of frame buffers in turn
        if ((st = ensure_ring(c)) != IQPT_OK) return st;
        if ((st = ensure_copy_stream(c)) != IQPT_OK) return st;
        // a gather in flight read an earlier ring buffer: keep the ring's reuse events in one order
        if (c->comm_pend) IQPT_HIP(hipStreamWaitEvent(c->stream3, c->ev_gend, 0));
        if (!c->end1) IQPT_HIP(hipEventRecord(c->ev_pipe_end, c->stream));
        if (!c->end2) IQPT_HIP(hipEventRecord(c->ev_s2, c->stream2));
        IQPT_HIP(hipStreamWaitEvent(c->stream3, c->end1 ? c->end1 : c->ev_pipe_end, 0));
        IQPT_HIP(hipStreamWaitEvent(c->stream3, c->end2 ? c->end2 : c->ev_s2, 0));
        if (wait) IQPT_HIP(hipStreamWaitEvent(c->stream3, wait, 0));
        IQPT_HIP(hipMemcpyAsync(dst, c->d_bgra, (size_t)c->npix * sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream3));
        c->copy_seq += 1;
        IQPT_HIP(hipEventRecord(c->pev[c->copy_seq % iqpt::kPipeRing], c->stream3));
        if (c->d_bgra == c->d_pring[c->pidx]) c->pseq[c->pidx] = c->copy_seq;
        *used = c->stream3;
        return IQPT_OK;
    }
    if (c->last_ovl && c->last_ls) {
        // overlapped launches in flight: copy on the last launch's stream without joining, so the next
        // launch still overlaps this one (from here on overlapped launches alternate two frame buffers)
        if (!c->d_bgra_alt) {
            if (hipMalloc(&c->d_bgra_alt, frame_words(c) * sizeof(uint32_t)) != hipSuccess) {
                (void)hipGetLastError();
                c->d_bgra_alt = nullptr;
                return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "second frame buffer for overlapped copies");
            }
            c->d_alt_own = c->d_bgra_alt;
        }
        cs = c->last_ls;
        if (cs == c->stream2) c->s2_pending = true;
    } else if ((st = join_streams(c)) != IQPT_OK) {
        return st;
    }
    if (wait) IQPT_HIP(hipStreamWaitEvent(cs, wait, 0));
    IQPT_HIP(hipMemcpyAsync(dst, c->d_bgra, (size_t)c->npix * sizeof(uint32_t), hipMemcpyDeviceToDevice, cs));
    *used = cs;
    return IQPT_OK;
}
}  // namespace

int iqpt_copy_frame_device_async(iqpt_ctx* c, void* dst_device, size_t bytes) {
    if (!c || !dst_device) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (bytes < (size_t)c->npix * sizeof(uint32_t)) return iqpt::fail(IQPT_ERR_INVALID_ARG, "destination too small");
    int st = use_device(c);
    if (st) return st;
    hipStream_t used = nullptr;
    return copy_frame_async(c, static_cast<uint32_t*>(dst_device), nullptr, &used);
}

int iqpt_frame_stream(iqpt_ctx* c, void** stream) {
    if (!c || !stream) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    // pipelined launches: the copy stream exists from the launch's end on (pipe_end), so the stream named
    // here is the one the next copy goes on (it used to appear only at the first copy)
    if (c->pipe) {
        int st = use_device(c);
        if (st) return st;
        if ((st = ensure_copy_stream(c)) != IQPT_OK) return st;
    }
    *stream = (void*)(c->pipe ? c->stream3 : ((c->last_ovl && c->last_ls) ? c->last_ls : c->stream));
    return IQPT_OK;
}

// ---- multi-GPU frame delivery over RCCL ----------------------------------

int iqpt_comm_unique_id(void* id, size_t bytes) {
    if (!id || bytes < IQPT_COMM_ID_BYTES) return iqpt::fail(IQPT_ERR_INVALID_ARG, "id NULL or shorter than IQPT_COMM_ID_BYTES");
    if (!rccl().get_unique_id) return iqpt::fail(IQPT_ERR_UNSUPPORTED, rccl().why);
    static_assert(sizeof(ncclUniqueId) == IQPT_COMM_ID_BYTES, "RCCL's unique id size");
    ncclUniqueId u;
    const ncclResult_t r = rccl().get_unique_id(&u);
    if (r != ncclSuccess) return rccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof u);
    return IQPT_OK;
}

int iqpt_comm_init(iqpt_ctx* c, int rank, int world, const void* id, size_t bytes) {
    if (!c || !id || bytes < IQPT_COMM_ID_BYTES) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument or short id");
    if (world < 1 || rank < 0 || rank >= world || (uint32_t)world > c->height)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "rank / world out of range");
    // the frame's cyclic row split (rank r owns rows r, r + S, ... of every column, S = the set's ystep), which
    // the root's assembly inverts: S = world on a node; S > world only for a one-GPU rehearsal of an S-way
    // share (the root then places the rows the communicator's ranks own)
    // (base = y0 - rank, the same on every rank: 0 on a node, rank 0's row offset in a rehearsal)
    const uint32_t split = c->set.ystep;
    const uint32_t nrows = (c->height - c->set.y0 + split - 1u) / split;
    if (c->set.x0 != 0 || c->set.x1 != c->width || c->set.y0 < (uint32_t)rank ||
        c->set.y0 - (uint32_t)rank + (uint32_t)world > split || c->set.nrows != nrows)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "the context's pixel set is not rank's cyclic rows of a world-way split "
                                                "(iqpt_pixel_set {0, W, rank, world, ceil((H - rank) / world)})");
    if (!rccl().comm_init_rank) return iqpt::fail(IQPT_ERR_UNSUPPORTED, rccl().why);
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    free_comm(c);
    const uint64_t stride = (uint64_t)((c->height + split - 1u) / split) * c->width;
    // the communicator's stream (its priority: iqpt_debug_set_gather; the lowest measured slower, r04 run 9:
    // the gather then finishes later and the double-buffered copies wait for it)
    int prio_least = 0, prio_greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) {
        (void)hipGetLastError();
        prio_least = prio_greatest = 0;
    }
    const int prio = c->gather_prio < 0 ? prio_least : (c->gather_prio > 0 ? prio_greatest : 0);
    if (hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, prio) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gcopy, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gend, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        free_comm(c);
        return iqpt::fail(IQPT_ERR_HIP, "communicator stream / events");
    }
    for (int i = 0; i < iqpt::kSendRing; ++i)
        if (hipMalloc(&c->d_gsend[i], stride * 16) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_gdone[i], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            free_comm(c);
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "gather send buffers");
        }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t comm = nullptr;
    // collective over the ranks; a frame of a few MB per rank needs few of RCCL's blocks, and every block
    // it runs takes a CU slot from the render kernels beside it (ncclConfig_t::maxCTAs)
    ncclResult_t r;
    if (c->gather_ctas > 0 && rccl().comm_init_config) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.minCTAs = 1;
        cfg.maxCTAs = c->gather_ctas;
        r = rccl().comm_init_config(&comm, world, u, rank, &cfg);
    } else {
        r = rccl().comm_init_rank(&comm, world, u, rank);
    }
    if (r != ncclSuccess) {
        free_comm(c);
        return rccl_fail(r, "ncclCommInitRank");
    }
    c->comm = comm;
    c->comm_rank = rank;
    c->comm_world = world;
    c->comm_stride = stride;
    c->gpar = 0;
    // the frame buffers pipelined launches write are the gather's send buffers as they are: pad every frame
    // buffer to the rank block. The last frame (d_bgra: the context's own buffer, the overlapped launches'
    // second one or a ring buffer) moves into the new own buffer; the second buffer, if there is one, is
    // re-made padded (the next overlapped launch overwrites it); a ring of the old size is dropped, rebuilt
    // at the next copy. (The views d_bgra / d_bgra_alt may point at any of these: none is kept.)
    if (stride > c->npix) {
        const size_t pbytes = (size_t)stride * sizeof(uint32_t);
        uint32_t* nb[2] = {};
        const int nbuf = c->d_alt_own ? 2 : 1;
        for (int k = 0; k < nbuf; ++k)
            if (hipMalloc(&nb[k], pbytes) != hipSuccess) {
                (void)hipGetLastError();
                for (uint32_t* b : nb)
                    if (b) (void)hipFree(b);
                free_comm(c);
                return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "padded frame buffer");
            }
        for (int k = 0; k < nbuf; ++k) IQPT_HIP(hipMemsetAsync(nb[k], 0, pbytes, c->stream));
        IQPT_HIP(hipMemcpyAsync(nb[0], c->d_bgra, (size_t)c->npix * sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
        IQPT_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_bgra_own);
        c->d_bgra_own = c->d_bgra = nb[0];
        if (c->d_alt_own) {
            (void)hipFree(c->d_alt_own);
            c->d_alt_own = c->d_bgra_alt = nb[1];
        }
        for (int i = 0; i < iqpt::kPipeRing; ++i) {
            if (c->d_pring[i]) (void)hipFree(c->d_pring[i]);
            c->d_pring[i] = nullptr;
            c->pseq[i] = 0;
        }
        c->pring_on = false;
        c->copy_seq = c->pwaited = 0;
    }
    return IQPT_OK;
}

namespace {
// One gather of `words` words per pixel (comm_stride pixels) from src to the root, assembled there into dst
// (W x H pixels), on cstream behind whatever it already waits for.
int gather_from(iqpt_ctx* c, const uint32_t* src, int root, uint32_t* dst, uint32_t words) {
    // timing (iqpt_comm_time): from the moment the send buffer is complete to the end of the root's assembly —
    // the transfer plus any wait for slower ranks inside the collective
    hipEvent_t t0 = take_event(c), t1 = take_event(c);
    if (t0) (void)hipEventRecord(t0, c->cstream);
    const bool is_root = root == c->comm_rank;
    if (is_root && !c->d_grecv) {
        if (hipMalloc(&c->d_grecv, (size_t)c->comm_world * c->comm_stride * 16) != hipSuccess) {
            (void)hipGetLastError();
            c->d_grecv = nullptr;
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "gather receive buffer");
        }
    }
    if (!(c->gather_skip & 1)) {
        const ncclResult_t r = rccl().gather(src, is_root ? c->d_grecv : nullptr,
                                             (size_t)c->comm_stride * words, ncclUint32, root,
                                             static_cast<ncclComm_t>(c->comm), c->cstream);
        if (r != ncclSuccess) return rccl_fail(r, "ncclGather");
    }
    if (is_root && !(c->gather_skip & 2)) {
        const int le = iqpt::launch_assemble_rows(c->cstream, c->d_grecv, dst, c->width, c->height,
                                                  (uint32_t)c->comm_world, c->set.ystep,
                                                  c->set.y0 - (uint32_t)c->comm_rank, c->comm_stride, words);
        if (le != 0) return iqpt::hip_fail((hipError_t)le, "frame assembly");
    }
    if (t1) (void)hipEventRecord(t1, c->cstream);
    if (t0 && t1) c->gtimed.emplace_back(t0, t1);
    IQPT_HIP(hipEventRecord(c->ev_gend, c->cstream));
    c->comm_pend = true;
    return IQPT_OK;
}

// ... from send buffer d_gsend[b], filled on stream `from`: behind that copy and nothing else
int gather_enqueue(iqpt_ctx* c, uint32_t b, hipStream_t from, int root, uint32_t* dst, uint32_t words) {
    IQPT_HIP(hipEventRecord(c->ev_gcopy, from));
    IQPT_HIP(hipStreamWaitEvent(c->cstream, c->ev_gcopy, 0));
    int st = gather_from(c, c->d_gsend[b], root, dst, words);
    if (st) return st;
    IQPT_HIP(hipEventRecord(c->ev_gdone[b], c->cstream));
    c->gdone_pend[b] = true;
    c->gpar = (b + 1u) % (uint32_t)iqpt::kSendRing;
    return IQPT_OK;
}

int comm_check(iqpt_ctx* c, int root) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (!c->comm) return iqpt::fail(IQPT_ERR_NOT_READY, "no communicator: call iqpt_comm_init first");
    if (root < 0 || root >= c->comm_world) return iqpt::fail(IQPT_ERR_INVALID_ARG, "root out of range");
    return use_device(c);
}

// Synchronous gather of the accumulators (what & 1) and / or the BGRA8 frame (what & 2) into d_gframe on the
// root (W x H x 4 words, reused for each); `out_lin` / `out_bgra` (root, host) receive them.
int gather_sync(iqpt_ctx* c, int root, int what, float* out_lin, uint8_t* out_bgra) {
    int st = enter(c);
    if (st) return st;
    const bool is_root = root == c->comm_rank;
    const size_t frame_px = (size_t)c->width * c->height;
    if (is_root && !c->d_gframe && hipMalloc(&c->d_gframe, frame_px * 16) != hipSuccess) {
        (void)hipGetLastError();
        c->d_gframe = nullptr;
        return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "assembled frame");
    }
    for (int k = 0; k < 2; ++k) {
        if (!(what & (1 << k))) continue;
        const uint32_t words = k == 0 ? 4u : 1u;
        const uint32_t b = c->gpar;
        if (c->gdone_pend[b]) IQPT_HIP(hipStreamWaitEvent(c->stream, c->ev_gdone[b], 0));
        if (k == 0) {
            const int le = iqpt::launch_relayout(c->stream, reinterpret_cast<const uint32_t*>(c->d_lin), c->d_gsend[b],
                                                 c->ncols, c->set.nrows, words, 1, true);
            if (le != 0) return iqpt::hip_fail((hipError_t)le, "gather copy");
        } else {
            IQPT_HIP(hipMemcpyAsync(c->d_gsend[b], c->d_bgra, (size_t)c->npix * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                    c->stream));            // the BGRA8 frame is compact already
        }
        if ((st = gather_enqueue(c, b, c->stream, root, c->d_gframe, words)) != IQPT_OK) return st;
        IQPT_HIP(hipStreamSynchronize(c->cstream));
        c->comm_pend = false;
        if (is_root && (k == 0 ? (void*)out_lin : (void*)out_bgra))
            IQPT_HIP(hipMemcpy(k == 0 ? (void*)out_lin : (void*)out_bgra, c->d_gframe, frame_px * words * 4,
                               hipMemcpyDeviceToHost));
    }
    IQPT_HIP(hipStreamSynchronize(c->stream));
    return check_dev_err(c);
}
}  // namespace

int iqpt_gather_frame_async(iqpt_ctx* c, int root, void* dst_device, size_t bytes) {
    int st = comm_check(c, root);
    if (st) return st;
    if (root == c->comm_rank && (!dst_device || bytes < (size_t)c->width * c->height * 4))
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "root: destination NULL or smaller than W x H x 4 bytes");
    if (c->pipe && c->d_bgra && !c->dev_err) {
        // pipelined launches: the launch's frame buffer (compact order, padded to the rank block) is the send
        // buffer — no copy: the communicator stream waits for the launch's kernels' own end events, gathers, and
        // records the ring's reuse event (the next launches writing this buffer wait for it, pipe_begin)
        if ((st = ensure_ring(c)) != IQPT_OK) return st;
        if (!c->end1) IQPT_HIP(hipEventRecord(c->ev_pipe_end, c->stream));
        if (!c->end2) IQPT_HIP(hipEventRecord(c->ev_s2, c->stream2));
        IQPT_HIP(hipStreamWaitEvent(c->cstream, c->end1 ? c->end1 : c->ev_pipe_end, 0));
        IQPT_HIP(hipStreamWaitEvent(c->cstream, c->end2 ? c->end2 : c->ev_s2, 0));
        // the ring's reuse events stay in one order whatever mixes copies (stream3) and gathers (cstream)
        if (c->copy_seq > 0) IQPT_HIP(hipStreamWaitEvent(c->cstream, c->pev[c->copy_seq % iqpt::kPipeRing], 0));
        if ((st = gather_from(c, c->d_bgra, root, static_cast<uint32_t*>(dst_device), 1u)) != IQPT_OK) return st;
        c->copy_seq += 1;
        IQPT_HIP(hipEventRecord(c->pev[c->copy_seq % iqpt::kPipeRing], c->cstream));
        if (c->d_bgra == c->d_pring[c->pidx]) c->pseq[c->pidx] = c->copy_seq;
        return IQPT_OK;
    }
    const uint32_t b = c->gpar;
    hipStream_t used = nullptr;
    // the copy into send buffer b waits for the gather that read it two gathers ago (long done)
    if ((st = copy_frame_async(c, c->d_gsend[b], c->gdone_pend[b] ? c->ev_gdone[b] : nullptr, &used)) != IQPT_OK)
        return st;
    return gather_enqueue(c, b, used, root, static_cast<uint32_t*>(dst_device), 1u);
}

int iqpt_gather_accum(iqpt_ctx* c, int root, void* dst_device, size_t bytes) {
    int st = comm_check(c, root);
    if (st) return st;
    const size_t need = (size_t)c->width * c->height * 16;
    if (root == c->comm_rank && (!dst_device || bytes < need))
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "root: destination NULL or smaller than W x H x 16 bytes");
    if ((st = enter(c)) != IQPT_OK) return st;
    const uint32_t b = c->gpar;
    if (c->gdone_pend[b]) IQPT_HIP(hipStreamWaitEvent(c->stream, c->ev_gdone[b], 0));
    const int le = iqpt::launch_relayout(c->stream, reinterpret_cast<const uint32_t*>(c->d_lin), c->d_gsend[b], c->ncols,
                                         c->set.nrows, 4, 1, true);
    if (le != 0) return iqpt::hip_fail((hipError_t)le, "gather copy");
    if ((st = gather_enqueue(c, b, c->stream, root, static_cast<uint32_t*>(dst_device), 4u)) != IQPT_OK) return st;
    IQPT_HIP(hipStreamSynchronize(c->cstream));
    c->comm_pend = false;
    return check_dev_err(c);
}

int iqpt_gather_read(iqpt_ctx* c, int root, float* lin_rgba, uint8_t* bgra) {
    int st = comm_check(c, root);
    if (st) return st;
    // every rank takes part in the same two gathers (the accumulators, then the BGRA8 frame) whatever the
    // root's pointers are: which collectives run cannot depend on one rank's arguments; the root's pointers
    // only choose what is copied back to the host (NULL: not copied)
    return gather_sync(c, root, IQPT_GATHER_ACCUM | IQPT_GATHER_FRAME, lin_rgba, bgra);
}

int iqpt_gather_read_select(iqpt_ctx* c, int root, int what, float* lin_rgba, uint8_t* bgra) {
    int st = comm_check(c, root);
    if (st) return st;
    if (what < 1 || what > (IQPT_GATHER_ACCUM | IQPT_GATHER_FRAME))
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "what must be IQPT_GATHER_ACCUM, IQPT_GATHER_FRAME or both");
    return gather_sync(c, root, what, lin_rgba, bgra);
}

int iqpt_comm_time(iqpt_ctx* c, double* total_ms, uint64_t* gathers) {
    if (!c || !total_ms || !gathers) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *total_ms = 0.0;
    *gathers = 0;
    if (!c->comm) return IQPT_OK;
    int st = use_device(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->cstream));
    double sum = 0.0;
    for (auto& g : c->gtimed) {
        float ms = 0.0f;
        IQPT_HIP(hipEventElapsedTime(&ms, g.first, g.second));
        sum += ms;
        c->event_pool.push_back(g.first);
        c->event_pool.push_back(g.second);
    }
    *total_ms = sum;
    *gathers = c->gtimed.size();
    c->gtimed.clear();
    return IQPT_OK;
}

int iqpt_comm_stream(iqpt_ctx* c, void** stream) {
    if (!c || !stream) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (!c->comm) return iqpt::fail(IQPT_ERR_NOT_READY, "no communicator: call iqpt_comm_init first");
    *stream = (void*)c->cstream;
    return IQPT_OK;
}

int iqpt_stream(iqpt_ctx* c, void** stream) {
    if (!c || !stream) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    *stream = (void*)c->stream;
    return IQPT_OK;
}

int iqpt_prepare(iqpt_ctx* c) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (!c->have_camera || !c->have_packet) return iqpt::fail(IQPT_ERR_NOT_READY, "camera and packet must be set");
    int st = enter(c);
    if (st) return st;
    if ((c->opt & iqpt::kOptPair) && (c->opt & iqpt::kOptCull) && (c->ntri + c->nsph) > 0 && !c->cull_valid &&
        (st = build_cull(c)) != IQPT_OK)
        return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    return IQPT_OK;
}

// kOptSplit statistics of the last launch (tools/split_share.py): split tiles, anchored tiles, split
// slots, leftovers of round 1, sum of the windows M, sum of the slots-per-sample estimates (x 256),
// split pixels, whether the last launch ran split. Synchronises.
int iqpt_debug_split_info(iqpt_ctx* c, unsigned long long* out8) {
    if (!c || !out8) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    for (int i = 0; i < 8; ++i) out8[i] = 0;
    out8[0] = c->n_split_tiles;
    out8[1] = c->n_anchor;
    const size_t ns = (size_t)c->n_split_tiles * iqpt::kQueueChunk;
    out8[2] = ns;
    // launch mode: 0 plain, 1 split, 5 split + fan, 6 spec (sphere pixels slot-parallel, the rest fan); 2-4 were the
    // chain and FAN launches (archived in round 6)
    out8[7] = c->spec_last ? 6 : (c->split_last ? (c->fan_last ? 5 : 1) : 0);
    if (!c->d_split || ns == 0) return IQPT_OK;
    uint32_t left = 0;
    IQPT_HIP(hipMemcpy(&left, c->d_queue + 2, sizeof left, hipMemcpyDeviceToHost));
    out8[3] = left;
    std::vector<uint32_t> v(3 * ns);
    IQPT_HIP(hipMemcpy(v.data(), c->d_split + c->n_anchor + c->n_split_tiles, v.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ns; ++i) {
        if (v[i] == ~0u) continue;
        out8[4] += v[ns + i];
        out8[5] += v[2 * ns + i];
        out8[6] += 1;
    }
    return IQPT_OK;
}

int iqpt_kernel_span(const iqpt_ctx* c, double* span_ms) {
    if (!c || !span_ms) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *span_ms = c->last_span_ms;
    return IQPT_OK;
}
int iqpt_set_overlap(iqpt_ctx* c, int mode) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (mode != IQPT_OVERLAP_OFF && mode != IQPT_OVERLAP_AUTO)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "overlap mode must be IQPT_OVERLAP_OFF or _AUTO");
    int st = enter(c);
    if (st) return st;
    c->overlap_mode = mode;
    return IQPT_OK;
}
int iqpt_set_split(iqpt_ctx* c, int mode) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    if (mode == IQPT_SPLIT_CHAIN || mode == IQPT_SPLIT_FAN)
        return iqpt::fail(IQPT_ERR_UNSUPPORTED, "CHAIN and FAN launches were archived in round 6 (branch round6-ab-archive)");
    if (mode != IQPT_SPLIT_AUTO && mode != IQPT_SPLIT_OFF && mode != IQPT_SPLIT_ON && mode != IQPT_SPLIT_SPEC)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "split mode must be IQPT_SPLIT_AUTO, _OFF, _ON or _SPEC");
    c->split_mode = mode;
    return IQPT_OK;
}

// The production option mask (kOptDefault) for A/B tools and tests.
int iqpt_debug_default_options(void) { return iqpt::kOptDefault; }

int iqpt_debug_set_kernel_options(iqpt_ctx* c, int opt) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    // (resident launches add kOptPrio when only that form is built, as iqpt_render does)
    if (!iqpt::render_variant_exists(c->max_depth, false, opt) &&
        !iqpt::render_variant_exists(c->max_depth, false, opt | iqpt::kOptPrio) &&
        !iqpt::render_variant_exists(c->max_depth, true, opt))
        return iqpt::fail(IQPT_ERR_UNSUPPORTED, "kernel option set not compiled into this build");
    int st = enter(c);
    if (st) return st;
    if ((opt & iqpt::kOptStats) && !c->d_stats) {
        const size_t words = iqpt::kStatsHeader + 3 * (size_t)iqpt::kStatsWaveSlots + iqpt::kStatsQueueSlots +
                             iqpt::kStatsPhaseWords * (size_t)iqpt::kStatsWaveSlots;
        if (hipMalloc(&c->d_stats, words * sizeof(unsigned long long)) != hipSuccess)
            return iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "stats");
        IQPT_HIP(hipMemset(c->d_stats, 0, words * sizeof(unsigned long long)));
    }
    c->opt = opt;
    c->opt_fixed = true;
    return IQPT_OK;
}

/* Internal (tests/test_cull.py): the host build of iq_interval.h for one tile of camera rays,
 * x in [xa, xb], y in [ya, yb]. tris: ntri x 9 floats (v0, e1, e2 world space); spheres: nsph x 4
 * (center, radius). Writes 1 per culled primitive; returns 0 with all flags 0 if the bundle is
 * unbounded (nothing can be culled). */
int iqpt_debug_cull_tile(const iqpt_camera* cam, uint32_t xa, uint32_t xb, uint32_t ya, uint32_t yb,
                         const float* tris, uint32_t ntri, const float* spheres, uint32_t nsph,
                         uint8_t* tri_culled, uint8_t* sph_culled) {
    if (!cam || (ntri && (!tris || !tri_culled)) || (nsph && (!spheres || !sph_culled)))
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    iqiv::camera_in ci;
    ci.width = cam->width;
    ci.height = cam->height;
    ci.rcp_width = 0.0f;
    ci.rcp_height = 0.0f;
    ci.inv_proj = cam->inv_proj;
    ci.inv_view = cam->inv_view;
    uint32_t cc = 0;
    cam_constants(*cam, &cc, &ci.near_rw, &ci.far_rw);
    ci.cam_const = (int)cc;
    const iqiv::bundle b = iqiv::camera_bundle(ci, xa, xb, ya, yb);
    for (uint32_t k = 0; k < ntri; ++k)
        tri_culled[k] = b.ok && iqiv::tri_culled(b, tris + 9 * k, tris + 9 * k + 3, tris + 9 * k + 6) ? 1 : 0;
    for (uint32_t k = 0; k < nsph; ++k) {
        const float* sp = spheres + 4 * k;
        sph_culled[k] = b.ok && iqiv::sphere_culled(b, sp, sp[3]) ? 1 : 0;
    }
    return b.ok ? 1 : 0;
}

/* Internal (tests/test_gpu_bvh.py): the BVH of the uploaded packet — node count and the number of
 * triangles left on the always-tested list (both 0 without a BVH). */
int iqpt_debug_bvh_info(iqpt_ctx* c, uint32_t* nnodes, uint32_t* nalways) {
    if (!c || !nnodes || !nalways) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *nnodes = c->d_bvh_nodes ? c->bvh_nnodes : 0u;
    *nalways = c->d_bvh_nodes ? c->bvh_nalways : 0u;
    return IQPT_OK;
}

/* Internal (tests/test_gpu_sphere_bvh.py): the sphere BVH of the uploaded packet — node count and the
 * number of spheres on the always-tested list (both 0 without one). */
int iqpt_debug_sbvh_info(iqpt_ctx* c, uint32_t* nnodes, uint32_t* nalways) {
    if (!c || !nnodes || !nalways) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *nnodes = c->d_sbvh_nodes ? c->sbvh_nnodes : 0u;
    *nalways = c->d_sbvh_nodes ? c->sbvh_nalways : 0u;
    return IQPT_OK;
}

/* Internal (tests/test_sphere_bvh.py): the sphere bound of iq_bvh.hpp, growth(S) for radii r_min,
 * r_max at origin distance S. */
double iqpt_debug_sphere_growth(double rmin, double rmax, double S) { return iqbvh::sphere_growth(rmin, rmax, S); }

/* Internal (tests/test_bvh.py): the error bound of iq_bvh.hpp for one triangle's edges, evaluated
 * at S = max_i |o_i - v0_i| and a lower bound D of the accepted determinant (D <= 1e-6: the reject
 * threshold). out: box growth, dt_a, dt_b (|t^ - t| <= dt_a + dt_b |t|), safety x E_det. Returns 1 if
 * the triangle is BVH-eligible, 0 if not. */
int iqpt_debug_bvh_bound(const float* e1, const float* e2, double S, double Md, double D, double* out4) {
    if (!e1 || !e2 || !out4) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    const iqbvh::tri_coeffs b = iqbvh::triangle_coeffs(e1, e2, Md);
    const double lambda = D > iqbvh::kDetMin ? iqbvh::kDetMin / D : 1.0;
    out4[0] = lambda * (b.gR + b.gB * S) + b.gC;
    out4[1] = lambda * b.tA * S;
    out4[2] = b.tB;
    out4[3] = b.edet;
    return b.eligible ? 1 : 0;
}

/* Internal (tests/test_gpu_libm.py): evaluate the device build of the shared math on n inputs on
 * the current device (synchronous). */
int iqpt_debug_libm(int fn, const float* a, const float* b, float* out, uint64_t n) {
    if (!a || !b || !out) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (n == 0) return IQPT_OK;
    if (n > (1ull << 28)) return iqpt::fail(IQPT_ERR_INVALID_ARG, "n too large");
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    const size_t bytes = (size_t)n * sizeof(float);
    int st = IQPT_OK;
    if (hipMalloc(&da, bytes) != hipSuccess || hipMalloc(&db, bytes) != hipSuccess ||
        hipMalloc(&dout, bytes) != hipSuccess) {
        st = iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "libm probe buffers");
    } else {
        hipError_t e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = (hipError_t)iqpt::launch_libm(nullptr, fn, da, db, dout, (uint32_t)n);
        if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) st = iqpt::hip_fail(e, "libm probe");
    }
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
    return st;
}

/* Internal (tests/test_camera_axis.py): 1 if the camera qualifies for the short pitch-only transform
 * (kOptCamAxis), its 16 launch constants in k16; 0 otherwise. Host only. */
int iqpt_debug_cam_axis(const iqpt_camera* cam, float* k16) {
    if (!cam || !k16) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    std::memset(k16, 0, 16 * sizeof(float));
    return cam_axis_constants(*cam, k16) ? 1 : 0;
}

/* Internal (tests/test_gpu_camera.py): the general camera transform and, if the camera qualifies,
 * the kOptCamAxis one, on the GPU for n (x_ndc, y_ndc) pairs; 6 floats (origin, direction) per ray
 * into gen / axis. Returns 1 if the axis form ran, 0 if not (synchronous). */
int iqpt_debug_camera_rays(const iqpt_camera* cam, const float* ndc, uint64_t n, float* gen, float* axis) {
    if (!cam || !ndc || !gen || !axis) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (n > (1ull << 24)) return iqpt::fail(IQPT_ERR_INVALID_ARG, "n too large");
    iqpt::kparams p;
    std::memset(&p, 0, sizeof p);
    p.width = cam->width;
    p.height = cam->height;
    std::memcpy(p.inv_proj, cam->inv_proj, sizeof p.inv_proj);
    std::memcpy(p.inv_view, cam->inv_view, sizeof p.inv_view);
    cam_constants(*cam, &p.cam_const, &p.cam_near_rw, &p.cam_far_rw);
    const bool ax = cam_axis_constants(*cam, p.cam_ax);
    if (n == 0) return ax ? 1 : 0;
    float *dn = nullptr, *dg = nullptr, *da = nullptr;
    int st = IQPT_OK;
    if (hipMalloc(&dn, n * 2 * sizeof(float)) != hipSuccess || hipMalloc(&dg, n * 6 * sizeof(float)) != hipSuccess ||
        hipMalloc(&da, n * 6 * sizeof(float)) != hipSuccess) {
        st = iqpt::fail(IQPT_ERR_OUT_OF_MEMORY, "camera probe buffers");
    } else {
        hipError_t e = hipMemcpy(dn, ndc, n * 2 * sizeof(float), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemset(da, 0, n * 6 * sizeof(float));
        if (e == hipSuccess) e = (hipError_t)iqpt::launch_camera_probe(nullptr, p, dn, dg, da, (uint32_t)n, ax);
        if (e == hipSuccess) e = hipMemcpy(gen, dg, n * 6 * sizeof(float), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(axis, da, n * 6 * sizeof(float), hipMemcpyDeviceToHost);
        if (e != hipSuccess) st = iqpt::hip_fail(e, "camera probe");
    }
    (void)hipFree(dn);
    (void)hipFree(dg);
    (void)hipFree(da);
    return st ? st : (ax ? 1 : 0);
}

/* Internal (tests/test_gpu_materials.py): set the frame counter (frames accumulated so far), e.g.
 * beyond 2^32 to exercise the running mean's large-n forms. */
int iqpt_debug_set_frame(iqpt_ctx* c, uint64_t frame) {
    if (!c) return iqpt::fail(IQPT_ERR_INVALID_ARG, "ctx is NULL");
    c->frame = frame;
    return IQPT_OK;
}

/* Internal (tests): the kernel option set of the context's last render launch (-1 before any), with bit 30 set when
 * that launch dealt its tiles to per-XCD lists and queue words (overlapped launches; streamed launches,
 * iqpt_debug_set_stream_xcd): the kernels fall back to one queue silently otherwise; bit 29 when it ran
 * iqpt_anyhit_kernel instead of the plain kernel (any-hit scenes with per-pixel masks on every tile). */
int iqpt_debug_last_options(iqpt_ctx* c, int* opt) {
    if (!c || !opt) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *opt = c->last_opt < 0 ? c->last_opt
                           : (c->last_opt | (c->last_xcd_lists ? (1 << 30) : 0) | (c->last_anyk ? (1 << 29) : 0));
    return IQPT_OK;
}

/* Internal (tools/wave_timeline.py): per wave slot of the last kOptStats launch, the shader-clock cycles spent in the
 * closest hits, the shading, the next rays and the rest of the loop (kStatsPhaseWords each, same slots as
 * iqpt_debug_read_wave_times). Call before iqpt_debug_read_stats. */
int iqpt_debug_read_wave_phases(iqpt_ctx* c, unsigned long long* out, uint32_t cap) {
    if (!c || !out) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    if (!c->d_stats) return iqpt::fail(IQPT_ERR_INVALID_ARG, "no stats buffer (kOptStats not set)");
    const size_t m = std::min<size_t>(cap, iqpt::kStatsWaveSlots);
    IQPT_HIP(hipMemcpy(out, c->d_stats + iqpt::kStatsHeader + 3 * (size_t)iqpt::kStatsWaveSlots + iqpt::kStatsQueueSlots,
                       iqpt::kStatsPhaseWords * m * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return IQPT_OK;
}

int iqpt_debug_read_wave_times(iqpt_ctx* c, unsigned long long* out, uint32_t cap, uint32_t* n) {
    if (!c || !out || !n) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *n = 0;
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    if (!c->d_stats) return IQPT_OK;
    unsigned long long cnt = 0;
    IQPT_HIP(hipMemcpy(&cnt, c->d_stats + 11, sizeof cnt, hipMemcpyDeviceToHost));
    const uint32_t m = (uint32_t)std::min<unsigned long long>({cnt, (unsigned long long)cap,
                                                               (unsigned long long)iqpt::kStatsWaveSlots});
    if (m) IQPT_HIP(hipMemcpy(out, c->d_stats + iqpt::kStatsHeader, 3 * (size_t)m * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost));
    *n = m;
    return IQPT_OK;
}

int iqpt_debug_read_stats(iqpt_ctx* c, unsigned long long* out16) {
    unsigned long long* out8 = out16;   // kStatsHeader (24) counters (tools/ab_kernel.py)
    if (!c || !out8) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    int st = enter(c);
    if (st) return st;
    IQPT_HIP(hipStreamSynchronize(c->stream));
    if (!c->d_stats) {
        std::memset(out8, 0, iqpt::kStatsHeader * sizeof(unsigned long long));
        return IQPT_OK;
    }
    IQPT_HIP(hipMemcpy(out8, c->d_stats, iqpt::kStatsHeader * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    IQPT_HIP(hipMemset(c->d_stats, 0, iqpt::kStatsHeader * sizeof(unsigned long long)));   // counters, wave slot index
    return IQPT_OK;
}

int iqpt_write_ppm(const char* path, uint32_t width, uint32_t height, const uint8_t* bgra) {
    if (!path || !bgra || !width || !height) return iqpt::fail(IQPT_ERR_INVALID_ARG, "bad PPM arguments");
    FILE* f = std::fopen(path, "wb");
    if (!f) return iqpt::fail(IQPT_ERR_INVALID_ARG, std::string("cannot open ") + path);
    std::fprintf(f, "P6\n%u %u\n255\n", width, height);
    std::vector<uint8_t> row((size_t)width * 3);
    for (uint32_t y = 0; y < height; ++y) {
        const uint8_t* src = bgra + (size_t)y * width * 4;
        for (uint32_t x = 0; x < width; ++x) {
            row[x * 3 + 0] = src[x * 4 + 2];
            row[x * 3 + 1] = src[x * 4 + 1];
            row[x * 3 + 2] = src[x * 4 + 0];
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    std::fclose(f);
    return IQPT_OK;
}

}  // extern "C"
