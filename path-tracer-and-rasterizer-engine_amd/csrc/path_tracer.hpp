// path_tracer.hpp — C++ facade with the reference's engine-plugin API over the iqpt C ABI.
//
// Mirrors IoniqRE's renderer_template (renderer_template.h:6-12) and path_tracer
// (path_tracer.h:12-67): the same singleton lifecycle (init(camera*) / shutdown() / get()), the
// same draw_scene(const scene&, std::vector<shader>&, float dt) cadence and deferred reset().
// The Direct3D present path (path_tracer.cu:171-210) is replaced by a headless PPM dump in
// end_frame(). Errors surface as iqpt::iqpt_exception carrying file/line and the C-ABI status,
// in the style of ioniq_exception / renderer_base::cuda_exception (ioniq_exception.h,
// renderer_base.cu:118-128).
#pragma once

#include <cstdint>
#include <exception>
#include <string>
#include <vector>

#include "iqpt.h"

namespace iqpt {

class iqpt_exception : public std::exception {
public:
    iqpt_exception(int line, const char* file, int status, std::string detail);
    const char* what() const noexcept override { return m_what.c_str(); }
    int status() const { return m_status; }

private:
    int m_status;
    std::string m_what;
};

#define IQPT_THROW_FAILED(call)                                                             \
    do {                                                                                    \
        int st_ = (call);                                                                   \
        if (st_ != IQPT_OK) throw ::iqpt::iqpt_exception(__LINE__, __FILE__, st_, iqpt_last_error()); \
    } while (0)

// The rasterizer's shader objects are accepted and ignored, as by the reference path tracer.
class shader {};

// camera (camera.h:8-34): host-side constructor + the matrices the kernel consumes.
class camera {
public:
    camera(uint16_t width, uint16_t height, float fovh = 45.0f, float znear = 0.01f, float zfar = 100.0f);
    uint16_t get_width() const { return m_cam.width; }
    uint16_t get_height() const { return m_cam.height; }
    const iqpt_camera& raw() const { return m_cam; }

private:
    iqpt_camera m_cam;
};

// scene (scene.h:17-104): name-keyed meshes and models, modified() flag, build_packet().
class scene {
public:
    scene();
    ~scene();
    scene(const scene&) = delete;
    scene& operator=(const scene&) = delete;

    void add_mesh_tri(const std::string& name);
    void add_mesh_quad(const std::string& name);
    void add_mesh_reg_polygon(const std::string& name, uint32_t vertices);
    void add_mesh_cube(const std::string& name);
    void add_mesh_uv_sphere(const std::string& name, bool flat = false, uint32_t segments = 32,
                            uint32_t rings = 16, iqpt_mesh_type t = IQPT_MESH_SPHERES);
    void add_model(const std::string& name, const std::string& mesh_name, const float scale[4],
                   const float rotation[4], const float translation[4]);
    void add_preset(const std::string& preset);

    bool modified() const { return m_modified; }
    // scene::build_packet (scene.cu:104-181) — host arrays; the upload is iqpt_upload_packet.
    iqpt_packet_desc build_packet() const;

private:
    iqpt_scene* m_scene = nullptr;
    mutable bool m_modified = true;
};

class renderer_template {                                                  // renderer_template.h:6-12
public:
    virtual ~renderer_template() = default;
    virtual void begin_frame() = 0;
    virtual void end_frame() = 0;
    virtual void draw_scene(const scene& scene, std::vector<shader>& shaders, float dt) = 0;
};

struct path_tracer_options {
    int device = 0;
    uint64_t seed = IQPT_DEFAULT_SEED;           // path_tracer.cu:45
    int max_depth = IQPT_DEFAULT_MAX_DEPTH;      // path_tracer.cu:240
    float launch_interval = 0.1f;                // path_tracer.cu:378
    uint32_t spp_per_launch = 1;                 // one sample per reference launch
    std::string ppm_path;                        // headless present target ("" = none)
    // multi-GPU (one process per GPU): this process renders rank's cyclic rows of the frame and the present
    // path gathers the frame to rank 0 over RCCL (iqpt_comm_init / iqpt_gather_read). comm_id: the bytes of
    // path_tracer::comm_unique_id() from one rank, shared out of band; empty = single GPU.
    int rank = 0;
    int world = 1;
    std::vector<uint8_t> comm_id;
};

class path_tracer : public renderer_template {
public:
    struct pixel {                                                         // path_tracer.h:14-20
        uint8_t b, g, r, a;
    };

    static void init(camera* cam, const path_tracer_options& opt = path_tracer_options());
    // an RCCL unique id for path_tracer_options::comm_id (made on one rank)
    static std::vector<uint8_t> comm_unique_id();
    static void shutdown();
    static path_tracer* get();

    void begin_frame() override;
    void end_frame() override;
    void draw_scene(const scene& scene, std::vector<shader>& shaders, float dt) override;
    void reset() { m_pending_reset = true; }                              // path_tracer.h:35

    // headless extensions; with a communicator the host frame is the whole gathered frame on rank 0
    const std::vector<pixel>& host_pixels() const { return m_host_pixels; }
    uint64_t frames() const;
    uint64_t rays_traced() const;
    void read_linear(std::vector<float>& rgba) const;
    // progressive accumulation checkpoint / resume (iqpt_checkpoint_save / _load)
    void save_checkpoint(const std::string& path) const;
    void load_checkpoint(const std::string& path);
    iqpt_ctx* context() const { return m_ctx; }

private:
    path_tracer(camera* cam, const path_tracer_options& opt);
    ~path_tracer() override;

    iqpt_ctx* m_ctx = nullptr;
    camera* m_camera;
    path_tracer_options m_opt;
    std::vector<pixel> m_host_pixels;
    float m_time = 0.0f;
    bool m_have_packet = false;
    bool m_image_updated = false;
    bool m_pending_reset = false;
    bool m_comm = false;          // rank's rows of a sharded frame (path_tracer_options::comm_id)
};

}  // namespace iqpt
