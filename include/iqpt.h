/*
 * iqpt.h — C ABI of the MI355X-native IoniqRE path tracer (libiqpt.so).
 *
 * This is the drop-in boundary for the reference's path-tracing hot path. Every entry point names
 * the reference interface it replaces (paths relative to the reference repo, IoniqRE/...):
 *
 *   reference                                              this ABI
 *   ---------------------------------------------------   ------------------------------------
 *   path_tracer::path_tracer / init (path_tracer.cu:48-142,
 *     path_tracer.h:24)  cudaMalloc fb/lin_fb/curandState
 *     + renderer_init_kernel (path_tracer.cu:36-46)        iqpt_create
 *   path_tracer::~path_tracer / shutdown (:144-164, :23)   iqpt_destroy
 *   camera::camera (camera.cu:5-18; managed memory,
 *     application.cu:16-17)                                iqpt_camera_init + iqpt_set_camera
 *   scene::build_packet upload half (scene.cu:183-233)
 *     and free_packet (scene.cu:238-264)                   iqpt_upload_packet
 *   render_kernel<<<>>> launch (path_tracer.cu:401-402,
 *     kernel :330-366), 1 sample per launch                iqpt_render (spp launches' worth)
 *   cudaDeviceSynchronize (path_tracer.cu:382)              iqpt_sync
 *   cudaMemcpy D2H of the BGRA frame (path_tracer.cu:385)   iqpt_read
 *   path_tracer::reset + deferred clear (path_tracer.h:35,
 *     path_tracer.cu:394-400)                              iqpt_reset
 *   D3D11 texture upload + Present (path_tracer.cu:171-210) iqpt_write_ppm (headless dump)
 *   RENDERER_THROW_CUDA / cuda_exception (renderer_base.h:14,
 *     renderer_base.cu:118-128)                            int status + iqpt_error_string /
 *                                                          iqpt_last_error
 *   scene / mesh / model builders (scene.cu:9-101,
 *     mesh.cu:66-279, model.cu:3-18)                       iqpt_scene_* (host only)
 *
 * Conventions: every function returns IQPT_OK (0) or an iqpt_status; nothing throws across the
 * ABI. Pointers are plain host pointers unless a name says "device". The library owns every
 * device allocation behind the opaque iqpt_ctx; caller buffers are only read (copied on upload)
 * or written (on read). One ctx per device per host thread; iqpt_render is asynchronous on the
 * ctx's own HIP stream, iqpt_read / iqpt_reset / iqpt_sync synchronise that stream.
 */
#ifndef IQPT_H
#define IQPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 6 (round 6): IQPT_SPLIT_CHAIN and IQPT_SPLIT_FAN are refused with IQPT_ERR_UNSUPPORTED (their kernels were
 * archived); the other entry points are unchanged from 5. */
#define IQPT_ABI_VERSION 6

typedef enum iqpt_status {
    IQPT_OK = 0,
    IQPT_ERR_INVALID_ARG = 1,   /* bad pointer, size, index or enum */
    IQPT_ERR_HIP = 2,           /* a HIP runtime call failed; iqpt_last_error() has the name */
    IQPT_ERR_OUT_OF_MEMORY = 3,
    IQPT_ERR_NO_DEVICE = 4,     /* no HIP device / device index out of range */
    IQPT_ERR_NOT_READY = 5,     /* render before camera/packet were set */
    IQPT_ERR_UNSUPPORTED = 6    /* e.g. max_depth above the compiled bound */
} iqpt_status;

/* ---------------------------------------------------------------- gpu_packet mirror */

/* mesh.h:12-26 `vertex` — AoS, 24 bytes. */
typedef struct iqpt_vertex {
    float pos[3];
    float normal[3];
} iqpt_vertex;

/* mesh.h:32-38 `mesh::type` */
typedef enum iqpt_mesh_type { IQPT_MESH_TRIANGLES = 0, IQPT_MESH_SPHERES = 1 } iqpt_mesh_type;

/* scene.h:26-31 `gpu_packet::tri_mesh` (host pointers here; the library copies them). */
typedef struct iqpt_tri_mesh {
    const iqpt_vertex* vertices;
    const uint32_t* indices;      /* clockwise triples */
    uint32_t num_indices;         /* must be a multiple of 3 */
    uint32_t num_vertices;
} iqpt_tri_mesh;

/* scene.h:33-37 `gpu_packet::tri_mesh_drawcall` — iqmat is row-vector, translation in row 3. */
typedef struct iqpt_tri_mesh_drawcall {
    float transform[16];          /* m[row][col] row-major, as iqmat::m (matrix.h:80) */
    uint32_t mesh_id;             /* index into tri_meshes */
} iqpt_tri_mesh_drawcall;

/* scene.h:38-42 `gpu_packet::sphere_drawcall` */
typedef struct iqpt_sphere_drawcall {
    float center[4];              /* iqvec; w ignored */
    float radius;
} iqpt_sphere_drawcall;

/* Per-primitive material table (README.txt:66-72 "planned"). The reference hard-wires
 * emissive(white, 10) on every triangle and oren_nayar(0.5, sigma 1) on every sphere
 * (path_tracer.cu:248-249, 278, 292); a packet without a table keeps exactly that. With a table,
 * every drawcall names one material, with the reference's two material classes (material.h:21-62):
 *   IQPT_MAT_EMISSIVE:   scatter = (albedo * param, cos 1, pdf 1), path ends (material.cu:50-57);
 *   IQPT_MAT_OREN_NAYAR: albedo, param = roughness sigma, clamped to [0, 1] like the constructor
 *                        (material.h:25-29); scatter as material.cu:5-48. On a triangle the hit normal
 *                        is the interpolated vertex normal, flipped to face the ray (shape.cu:93-101). */
#define IQPT_MAT_EMISSIVE 0u
#define IQPT_MAT_OREN_NAYAR 1u
typedef struct iqpt_material {
    uint32_t type;                /* IQPT_MAT_* */
    float albedo[4];              /* iqvec color (w unused by the output) */
    float param;                  /* emissive: strength; Oren-Nayar: roughness sigma */
} iqpt_material;

/* scene.h:21-45 `scene::gpu_packet` with host pointers, plus the optional material table. */
typedef struct iqpt_packet_desc {
    uint32_t num_drawcalls[2];    /* [IQPT_MESH_TRIANGLES], [IQPT_MESH_SPHERES] */
    uint32_t num_tri_meshes;
    const iqpt_tri_mesh* tri_meshes;
    const iqpt_tri_mesh_drawcall* tri_mesh_dcs;
    const iqpt_sphere_drawcall* sphere_dcs;
    /* NULL = the reference's materials. Otherwise num_materials entries and one index per drawcall. */
    const iqpt_material* materials;
    uint32_t num_materials;
    const uint32_t* tri_dc_material;      /* [num_drawcalls[IQPT_MESH_TRIANGLES]] */
    const uint32_t* sphere_dc_material;   /* [num_drawcalls[IQPT_MESH_SPHERES]] */
} iqpt_packet_desc;

/* camera.h:22-32 `camera` layout (uint16 size, fov, position/forward, 4 matrices). */
typedef struct iqpt_camera {
    uint16_t width;
    uint16_t height;
    float fovh;                   /* degrees */
    float position[4];
    float forward[4];
    float view[16];
    float projection[16];
    float inv_view[16];
    float inv_proj[16];
} iqpt_camera;

/* Which pixels of the W x H frame a ctx owns: columns [x0, x1), rows y0 + k*ystep for k < nrows.
 * The RNG stream and the camera ray of a pixel are keyed by its GLOBAL id y*W + x
 * (path_tracer.cu:43,338), so any partition renders bit-identical pixels. Device buffers are
 * compact: pixel (col c, row k) of the set is element k*(x1-x0) + c. */
typedef struct iqpt_pixel_set {
    uint32_t x0, x1;
    uint32_t y0, ystep, nrows;
} iqpt_pixel_set;

/* Defaults of the reference (camera.h:11, path_tracer.cu:45, path_tracer.cu:240). */
#define IQPT_DEFAULT_SEED 1984ull
#define IQPT_DEFAULT_MAX_DEPTH 5
#define IQPT_MAX_DEPTH_LIMIT 16

typedef struct iqpt_ctx iqpt_ctx;

/* camera::camera(width, height, fovh, znear, zfar) (camera.cu:5-18): builds view = look_at(
 * position, position + forward), projection = perspective(W/H, radians(fovh), znear, zfar) and
 * their inverses with the reference's matrix code (matrix.cu). position/forward default to the
 * reference's (0,.5,-3,0)/(0,-.5,3,0) (camera.h:26-27); pass NULL to keep them. Host only. */
int iqpt_camera_init(iqpt_camera* cam, uint16_t width, uint16_t height, float fovh_deg,
                     float znear, float zfar, const float position[4], const float forward[4]);

/* Creates a render context on HIP device `device` for a width x height frame. `pixels` selects
 * the owned subset (NULL = the whole frame). Allocates the accumulator (float4), the BGRA8 frame
 * and the per-pixel XORWOW states and runs the RNG init kernel: curand_init(seed, pixelid, 0). */
int iqpt_create(int device, uint32_t width, uint32_t height, const iqpt_pixel_set* pixels,
                uint64_t seed, int max_depth, iqpt_ctx** out);
int iqpt_destroy(iqpt_ctx* ctx);

int iqpt_set_camera(iqpt_ctx* ctx, const iqpt_camera* cam);

/* Copies the packet and re-lays it out for the kernel: triangles flattened over drawcalls in
 * packet order, positions pre-transformed to world space and edges precomputed with the
 * reference's exact operation order (the per-ray transforms of path_tracer.cu:257-270 are
 * ray-independent), spheres SoA. Rejects mesh_id / index out of range. */
int iqpt_upload_packet(iqpt_ctx* ctx, const iqpt_packet_desc* packet);

/* Renders `spp` samples per owned pixel: bit-identical to `spp` consecutive reference launches
 * (same RNG consumption, same running-mean formula, frame counter continues). Asynchronous. */
int iqpt_render(iqpt_ctx* ctx, uint32_t spp);
int iqpt_sync(iqpt_ctx* ctx);

/* Sample-parallel chains (no reference counterpart: the reference runs one sample per
 * pixel per launch, path_tracer.cu:330-366). A pixel's samples are one sequential XORWOW stream
 * (path_tracer.cu:339), so its samples cannot simply be spread over threads; in split mode the pixels
 * whose camera rays may scatter have a sample evaluated at every even stream offset of a window in
 * parallel, then the chain is stitched in order — bit-identical results, more parallelism when a
 * context owns few pixels (a row share of a multi-GPU frame). AUTO (the default) splits when the
 * owned pixels are few per resident GPU lane; ON / OFF force it (resident scenes only). */
#define IQPT_SPLIT_AUTO (-1)
#define IQPT_SPLIT_OFF 0
#define IQPT_SPLIT_ON 1
/* CHAIN and FAN were launch modes of rounds 2-5, archived in round 6 (AUTO never chose
 * FAN, and CHAIN only where SPEC did not fit): iqpt_set_split refuses them with IQPT_ERR_UNSUPPORTED. */
#define IQPT_SPLIT_CHAIN 2
#define IQPT_SPLIT_FAN 3
/* SPEC: the pixels whose own camera rays may reach a sphere (the only ones whose samples
 * take more than two draws) have every slot of a window evaluated in parallel and their chains walked in
 * order afterwards; every other pixel's samples are spread over the four waves of a tile's block of the fan
 * kernel (every sample one ray and two draws, so sample k starts 2k draws into the pixel's stream) and
 * folded in order, on a second stream, the two kernels pipelined across launches. AUTO picks it for small
 * shares (fewer than 4 owned pixels per resident lane: C3 at N >= 2). */
#define IQPT_SPLIT_SPEC 4
int iqpt_set_split(iqpt_ctx* ctx, int mode);

/* Overlapped launches (no reference counterpart: the reference launches one frame at a
 * time on one stream, path_tracer.cu:370-392). With AUTO (the default) consecutive iqpt_render calls on
 * a resident scene alternate between two HIP streams, so a launch starts filling the CUs its
 * predecessor's tail leaves idle; each screen tile is bound to one XCD and waits, per tile, until the
 * previous launch has finished it — bit-identical results. Every other call joins the streams. OFF
 * renders every launch on one stream. */
#define IQPT_OVERLAP_OFF 0
#define IQPT_OVERLAP_AUTO 1
int iqpt_set_overlap(iqpt_ctx* ctx, int mode);

/* Builds the per-view acceleration state (the tile masks, queue order and split set of the current
 * camera and packet) now instead of inside the next iqpt_render, and synchronises: lets a caller time
 * the setup the reference pays on every scene change (path_tracer.cu:389-392). Optional. */
int iqpt_prepare(iqpt_ctx* ctx);

/* path_tracer::reset: the next sample restarts the running mean at frame 1 and the BGRA frame is
 * cleared; the accumulator and RNG states are kept, exactly as the reference (path_tracer.cu:394-400). */
int iqpt_reset(iqpt_ctx* ctx);

/* Synchronises and copies out the owned pixels (compact order). Either pointer may be NULL.
 * lin_rgba: 4 floats per pixel (the reference's iqvec lin_fb; w is never written by the kernel).
 * bgra: 4 bytes per pixel, B,G,R,A (path_tracer.h:14-20). */
int iqpt_read(iqpt_ctx* ctx, float* lin_rgba, uint8_t* bgra);
/* XORWOW states, 6 words per pixel: v[0..4], d. */
int iqpt_read_rng(iqpt_ctx* ctx, uint32_t* states);
/* Device-to-device copy of the accumulator (npix float4) into a caller device buffer on the
 * ctx's stream (used by the multi-GPU gather). Synchronises. */
int iqpt_copy_accum_device(iqpt_ctx* ctx, void* dst_device, size_t bytes);
/* Device-to-device copy of the BGRA8 frame (npix uint32, compact order) into a caller device buffer:
 * the multi-GPU gather of the presented frame (path_tracer.cu:385 reads this buffer back every
 * frame). Synchronises. */
int iqpt_copy_frame_device(iqpt_ctx* ctx, void* dst_device, size_t bytes);
/* Stream-ordered form of iqpt_copy_frame_device for a pipelined gather: the copy is enqueued after
 * every render issued so far, on the stream iqpt_frame_stream names, and the call returns at once (no
 * host sync). It does not join overlapped or pipelined launches: the next render still overlaps the last
 * one (from the first such copy on, those launches write the frame into two buffers in turn, DESIGN.md §7,
 * §3.11). The caller orders its own work against iqpt_frame_stream's stream, asked right before this call. */
int iqpt_copy_frame_device_async(iqpt_ctx* ctx, void* dst_device, size_t bytes);
/* The context's HIP stream (hipStream_t): renders, and every copy out, are ordered on it (overlapped
 * launches join it before any other call but iqpt_copy_frame_device_async). */
int iqpt_stream(iqpt_ctx* ctx, void** stream);
/* The stream iqpt_copy_frame_device_async enqueues on now: that of the last render launch while
 * overlapped launches are in flight, a copy stream behind both kernels of the last launch while
 * pipelined spec launches are (IQPT_SPLIT_SPEC), else the context's stream. Work enqueued there runs after
 * that launch, not after the ones issued later. */
int iqpt_frame_stream(iqpt_ctx* ctx, void** stream);

/* ---------------------------------------------------------------- multi-GPU frame delivery
 * One process per GPU, one ctx per process, each owning its rank's cyclic rows of ONE frame: pixel set
 * {0, W, rank, world, ceil((H - rank) / world)} (row y -> rank y mod world; the RNG stream and camera ray of a
 * pixel are keyed by its global id, path_tracer.cu:36-46 and :336-339, so the assembled frame is bit-identical
 * to one GPU's). The frame the reference copies back after every launch (path_tracer.cu:385, the D3D present
 * of :171-210) is gathered to a root rank over RCCL (ncclGather over xGMI) and assembled there
 * in row-major order. The reference is single-GPU; these calls are the library's multi-GPU extension of
 * that readback. RCCL is loaded at the first call (librccl.so.1; a process that already holds one, e.g.
 * PyTorch-ROCm's, shares it).
 *
 * iqpt_comm_unique_id: on one rank, then handed to every rank out of band (MPI, a TCP store, a file).
 * iqpt_comm_init: collective over the world ranks (each blocks until all have called it); fails with
 *   IQPT_ERR_INVALID_ARG unless the ctx owns exactly its rank's cyclic rows {0, W, rank, S, ceil((H - rank) / S)}
 *   with S >= world (S = world on a node; S > world is a rehearsal of an S-way share on fewer GPUs, in which
 *   the root places the rows of the communicator's ranks only).
 * iqpt_gather_frame_async: collective; enqueues a copy of the BGRA8 frame behind every render issued so far
 *   (it does not end overlapped or pipelined launches, like iqpt_copy_frame_device_async; after a pipelined
 *   launch no copy: the gather reads the frame buffer the launch wrote, behind its kernels), the gather and,
 *   on the root, the assembly of the W x H frame into dst_device (W*H*4 bytes; ignored elsewhere) on the
 *   communicator's stream (iqpt_comm_stream), and returns. The caller orders its reads of dst_device on that
 *   stream; every other entry point waits for the gathers in flight.
 * iqpt_gather_accum: collective, synchronous; the float4 accumulators (W*H*16 bytes of device memory) on the root.
 * iqpt_gather_read: collective, synchronous; the whole frame's accumulator (W*H*4 floats) and BGRA8 (W*H*4
 *   bytes) into the root's host buffers (either may be NULL; other ranks' pointers are ignored) — the
 *   multi-GPU iqpt_read. Both planes cross the interconnect on every call.
 * iqpt_gather_read_select: the same for the planes in `what` only (IQPT_GATHER_ACCUM | IQPT_GATHER_FRAME; every
 *   rank passes the same value, the collectives must match): a present that needs the BGRA8 frame alone moves
 *   4 instead of 20 bytes per pixel. */
#define IQPT_COMM_ID_BYTES 128
int iqpt_comm_unique_id(void* id, size_t bytes);
int iqpt_comm_init(iqpt_ctx* ctx, int rank, int world, const void* id, size_t bytes);
int iqpt_gather_frame_async(iqpt_ctx* ctx, int root, void* dst_device, size_t bytes);
int iqpt_gather_accum(iqpt_ctx* ctx, int root, void* dst_device, size_t bytes);
int iqpt_gather_read(iqpt_ctx* ctx, int root, float* lin_rgba, uint8_t* bgra);
#define IQPT_GATHER_ACCUM 1
#define IQPT_GATHER_FRAME 2
int iqpt_gather_read_select(iqpt_ctx* ctx, int root, int what, float* lin_rgba, uint8_t* bgra);
int iqpt_comm_stream(iqpt_ctx* ctx, void** stream);
/* Sum of the gathers' durations on the communicator's stream (from the rank's copy being done to the end
 * of the gather and, on the root, of the assembly: the transfer plus any wait for slower ranks) and their
 * count, since the last call (then cleared). Synchronises the communicator's stream. */
int iqpt_comm_time(iqpt_ctx* ctx, double* total_ms, uint64_t* gathers);

int iqpt_num_pixels(const iqpt_ctx* ctx, uint64_t* npix);
int iqpt_frame_count(const iqpt_ctx* ctx, uint64_t* frames);
/* Closest-hit queries (rays) traced since creation (Σ final crt_depth, path_tracer.cu:252-318). Synchronises. */
int iqpt_rays_traced(iqpt_ctx* ctx, uint64_t* rays);
/* Sum of the render-kernel durations measured with HIP events on the ctx stream, and the number
 * of launches, since the last call (then cleared). Synchronises. */
int iqpt_kernel_time(iqpt_ctx* ctx, double* total_ms, uint64_t* launches);
/* The launches of the last iqpt_kernel_time call from the first one's start to the last one's end
 * (equal to total_ms for launches that did not overlap, less when they did). */
int iqpt_kernel_span(const iqpt_ctx* ctx, double* span_ms);
/* Name of the render kernel as it appears in rocprofv3 traces. */
const char* iqpt_kernel_name(void);

/* Checkpoint / resume of the progressive accumulation (the reference keeps this
 * state only in device memory, path_tracer.cu:129-141). The file holds everything a context carries
 * between launches — accumulator, BGRA frame, XORWOW states, frame counter, rays traced — so that
 * render(a); checkpoint_save; ... checkpoint_load into a context created with the same frame size,
 * pixel set, seed and max_depth; render(b) is bit-identical to render(a + b) in one context.
 * Save synchronises and writes atomically (temporary file + rename); load validates the header, the
 * sizes and an FNV-1a checksum before touching the context (IQPT_ERR_INVALID_ARG otherwise). */
int iqpt_checkpoint_save(iqpt_ctx* ctx, const char* path);
int iqpt_checkpoint_load(iqpt_ctx* ctx, const char* path);

/* Headless replacement of the D3D11 present path: writes a binary PPM (P6) from BGRA8 pixels. */
int iqpt_write_ppm(const char* path, uint32_t width, uint32_t height, const uint8_t* bgra);

const char* iqpt_error_string(int status);
/* Detail of the last failure on this thread (HIP error name/description, argument checked). */
const char* iqpt_last_error(void);
int iqpt_abi_version(void);

/* ---------------------------------------------------------------- scene builder (host only)
 * Mirrors scene / mesh / model (scene.h:17-104, mesh.h:28-94, model.h:8-41): name-keyed meshes
 * and models; build_packet walks models sorted by mesh name and assigns mesh_id by lower_bound
 * over ALL mesh names (scene.cu:161-181) — including the reference's quirk that mesh_id indexes
 * the uncompacted name list. Models that share a mesh are ordered by insertion (the reference
 * orders them by heap address, scene.h:58-67, which is not reproducible). */
typedef struct iqpt_scene iqpt_scene;

int iqpt_scene_create(iqpt_scene** out);
int iqpt_scene_destroy(iqpt_scene* s);
/* Procedural meshes of mesh.cu: tri (:66-80), quad (:82-98), reg_polygon (:100-128),
 * cube (:130-186), uv_sphere (:190-279). */
int iqpt_scene_add_mesh_tri(iqpt_scene* s, const char* name);
int iqpt_scene_add_mesh_quad(iqpt_scene* s, const char* name);
int iqpt_scene_add_mesh_reg_polygon(iqpt_scene* s, const char* name, uint32_t vertices);
int iqpt_scene_add_mesh_cube(iqpt_scene* s, const char* name);
int iqpt_scene_add_mesh_uv_sphere(iqpt_scene* s, const char* name, int flat, uint32_t segments,
                                  uint32_t rings, int mesh_type);
int iqpt_scene_add_mesh(iqpt_scene* s, const char* name, int mesh_type,
                        const iqpt_vertex* vertices, uint32_t num_vertices,
                        const uint32_t* indices, uint32_t num_indices);
/* model::set_transforms(scale, rotation, translation) (model.cu:3-9): transform =
 * scale * rotation_x * rotation_y * rotation_z * translate (model.cu:11-18). */
int iqpt_scene_add_model(iqpt_scene* s, const char* name, const char* mesh_name,
                         const float scale[4], const float rotation[4], const float translation[4]);
int iqpt_scene_num_meshes(const iqpt_scene* s, uint32_t* n);
/* Scenes of BASELINE.json's configs, built with the calls above:
 *   "app_default" application.cu:25-34, "c1_plumbing" C1, "cornell" C2/C3, "mesh10k" C4, "mixed" C5. */
int iqpt_scene_add_preset(iqpt_scene* s, const char* preset);
/* Material table of the scene builder: add a material (its index is returned) and assign it to a
 * model; the packet carries a table as soon as one material was added (models without an assignment
 * then get the reference's default for their mesh type: emissive(white, 10) for triangle meshes,
 * oren_nayar(0.5, 1) for spheres). */
int iqpt_scene_add_material(iqpt_scene* s, const iqpt_material* m, uint32_t* index);
int iqpt_scene_set_model_material(iqpt_scene* s, const char* model, uint32_t material);
/* Builds the packet into arrays owned by the scene (valid until the next build or destroy). */
int iqpt_scene_build_packet(iqpt_scene* s, iqpt_packet_desc* out);

#ifdef __cplusplus
}
#endif

#endif /* IQPT_H */
