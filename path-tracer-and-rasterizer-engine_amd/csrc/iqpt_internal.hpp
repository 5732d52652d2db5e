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

// Device layout of one triangle for the intersection loop: 3 x float4 = 48 B,
//   t0 = (v0.x, v0.y, v0.z, e1.x), t1 = (e1.y, e1.z, e2.x, e2.y), t2 = (e2.z, 0, 0, 0)
// where v0 is the world-space first vertex and e1 = v1 - v0, e2 = v2 - v0 (shape.cu:65-66).
constexpr int kTriFloat4 = 3;
// Shading record per triangle (only read for the closest hit): world normals n0, n1, n2 and the
// geometric normal e1 x e2 (shape.cu:96-101) packed in the w lanes — 3 x float4. Not read under the reference's
// hard-wired materials (every triangle is emissive, path_tracer.cu:278), kept for the
// per-primitive material table.
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
    const float4_storage* tris;      // ntri * kTriFloat4
    uint32_t ntri;
    const float4_storage* spheres;   // nsph * (center.xyz, radius)
    uint32_t nsph;
    uint32_t tri_batch;              // triangles staged in LDS per batch
    uint32_t sph_batch;              // spheres staged in LDS per batch
    float4_storage* lin;             // npix
    uint32_t* bgra;                  // npix
    uint32_t* rng;                   // 6 planes of npix words: v0..v4, d
    unsigned long long* rays;        // closest-hit query counter
    uint32_t* queue;                 // pixel dequeue head (zeroed before every launch)
};

// Launch wrappers (iqpt_kernels.hip). Return a hipError_t as int.
int launch_rng_init(void* stream, uint32_t width, uint32_t x0, uint32_t ncols, uint32_t y0,
                    uint32_t ystep, uint32_t npix, uint64_t seed, const uint32_t* tables,
                    uint32_t* rng);
// grid_blocks = persistent grid size; lds_bytes dynamic LDS; stream = hipStream_t.
int launch_render(void* stream, const kparams& p, uint32_t grid_blocks, uint32_t lds_bytes, bool stream_batches);
// Max resident blocks per CU of the render kernel for the given dynamic LDS (occupancy query).
int render_occupancy(int max_depth, bool stream_batches, uint32_t lds_bytes, int* blocks_per_cu);
constexpr int kRenderBlock = 256;
constexpr uint32_t kQueueChunk = 64;
const char* render_kernel_name();

}  // namespace iqpt
