// path_tracer.cpp — the facade of path_tracer.hpp (IoniqRE/path_tracer.cu:16-34, 48-210, 368-404).
#include "path_tracer.hpp"

#include <sstream>
#include <utility>

namespace iqpt {

namespace {
path_tracer* g_path_tracer = nullptr;                                      // path_tracer.cu:12
}

iqpt_exception::iqpt_exception(int line, const char* file, int status, std::string detail) : m_status(status) {
    std::ostringstream oss;
    oss << "Ioniq Path Tracer Exception\n"
        << "[Error Code]: " << status << "\n"
        << "[Name]: " << iqpt_error_string(status) << "\n"
        << "[Description]: " << detail << "\n"
        << "[File]: " << file << "\n[Line]: " << line;
    m_what = oss.str();
}

camera::camera(uint16_t width, uint16_t height, float fovh, float znear, float zfar) {
    IQPT_THROW_FAILED(iqpt_camera_init(&m_cam, width, height, fovh, znear, zfar, nullptr, nullptr));
}

scene::scene() { IQPT_THROW_FAILED(iqpt_scene_create(&m_scene)); }
scene::~scene() { iqpt_scene_destroy(m_scene); }

void scene::add_mesh_tri(const std::string& n) { IQPT_THROW_FAILED(iqpt_scene_add_mesh_tri(m_scene, n.c_str())); }
void scene::add_mesh_quad(const std::string& n) { IQPT_THROW_FAILED(iqpt_scene_add_mesh_quad(m_scene, n.c_str())); }
void scene::add_mesh_reg_polygon(const std::string& n, uint32_t v) {
    IQPT_THROW_FAILED(iqpt_scene_add_mesh_reg_polygon(m_scene, n.c_str(), v));
}
void scene::add_mesh_cube(const std::string& n) { IQPT_THROW_FAILED(iqpt_scene_add_mesh_cube(m_scene, n.c_str())); }
void scene::add_mesh_uv_sphere(const std::string& n, bool flat, uint32_t segments, uint32_t rings, iqpt_mesh_type t) {
    IQPT_THROW_FAILED(iqpt_scene_add_mesh_uv_sphere(m_scene, n.c_str(), flat ? 1 : 0, segments, rings, (int)t));
}
void scene::add_model(const std::string& name, const std::string& mesh_name, const float scale[4],
                      const float rotation[4], const float translation[4]) {
    IQPT_THROW_FAILED(iqpt_scene_add_model(m_scene, name.c_str(), mesh_name.c_str(), scale, rotation, translation));
    m_modified = true;                                                     // scene.cu:49
}
void scene::add_preset(const std::string& preset) {
    IQPT_THROW_FAILED(iqpt_scene_add_preset(m_scene, preset.c_str()));
    m_modified = true;
}
iqpt_packet_desc scene::build_packet() const {
    iqpt_packet_desc pk{};
    m_modified = false;                                                    // scene.cu:112
    IQPT_THROW_FAILED(iqpt_scene_build_packet(m_scene, &pk));
    return pk;
}

void path_tracer::init(camera* cam, const path_tracer_options& opt) {     // path_tracer.cu:16-21
    if (!g_path_tracer) g_path_tracer = new path_tracer(cam, opt);
}
void path_tracer::shutdown() {                                             // path_tracer.cu:23-29
    delete g_path_tracer;
    g_path_tracer = nullptr;
}
path_tracer* path_tracer::get() { return g_path_tracer; }

std::vector<uint8_t> path_tracer::comm_unique_id() {
    std::vector<uint8_t> id(IQPT_COMM_ID_BYTES);
    IQPT_THROW_FAILED(iqpt_comm_unique_id(id.data(), id.size()));
    return id;
}

path_tracer::path_tracer(camera* cam, const path_tracer_options& opt) : m_camera(cam), m_opt(opt) {
    const uint32_t w = cam->get_width(), h = cam->get_height();
    if (opt.comm_id.empty()) {
        IQPT_THROW_FAILED(iqpt_create(opt.device, w, h, nullptr, opt.seed, opt.max_depth, &m_ctx));
    } else {
        // rank's cyclic rows of the frame (row y -> rank y mod world), then the communicator (collective)
        const uint32_t r = (uint32_t)opt.rank, n = (uint32_t)opt.world;
        const iqpt_pixel_set rows{0, w, r, n, n && r < h ? (h - r + n - 1) / n : 0};
        IQPT_THROW_FAILED(iqpt_create(opt.device, w, h, &rows, opt.seed, opt.max_depth, &m_ctx));
        IQPT_THROW_FAILED(iqpt_comm_init(m_ctx, opt.rank, opt.world, opt.comm_id.data(), opt.comm_id.size()));
        m_comm = true;
    }
    IQPT_THROW_FAILED(iqpt_set_camera(m_ctx, &cam->raw()));
    m_host_pixels.assign((size_t)w * h, pixel{0, 0, 0, 0});              // path_tracer.cu:130-131
}

path_tracer::~path_tracer() { iqpt_destroy(m_ctx); }

void path_tracer::begin_frame() {}

void path_tracer::end_frame() {                                            // path_tracer.cu:171-210
    if (m_image_updated && !m_opt.ppm_path.empty() && m_opt.rank == 0) {
        IQPT_THROW_FAILED(iqpt_write_ppm(m_opt.ppm_path.c_str(), m_camera->get_width(), m_camera->get_height(),
                                         reinterpret_cast<const uint8_t*>(m_host_pixels.data())));
    }
    m_image_updated = false;
}

void path_tracer::draw_scene(const scene& scn, std::vector<shader>& /*shaders*/, float dt) {  // :368-404
    m_time += dt;
    if (!(m_time > m_opt.launch_interval)) return;
    m_time = 0.0f;
    // sync with the previous launch and fetch its frame (:382-386); sharded: the whole frame on rank 0
    uint8_t* host = reinterpret_cast<uint8_t*>(m_host_pixels.data());
    if (m_comm) IQPT_THROW_FAILED(iqpt_gather_read_select(m_ctx, 0, IQPT_GATHER_FRAME, nullptr, host));
    else IQPT_THROW_FAILED(iqpt_read(m_ctx, nullptr, host));
    m_image_updated = true;
    if (scn.modified() || !m_have_packet) {                                // :389-392
        const iqpt_packet_desc pk = scn.build_packet();
        IQPT_THROW_FAILED(iqpt_upload_packet(m_ctx, &pk));
        m_have_packet = true;
    }
    if (m_pending_reset) {                                                 // :394-400
        IQPT_THROW_FAILED(iqpt_reset(m_ctx));
        m_pending_reset = false;
    }
    IQPT_THROW_FAILED(iqpt_render(m_ctx, m_opt.spp_per_launch));          // :401-402
}

uint64_t path_tracer::frames() const {
    uint64_t f = 0;
    IQPT_THROW_FAILED(iqpt_frame_count(m_ctx, &f));
    return f;
}

uint64_t path_tracer::rays_traced() const {
    uint64_t r = 0;
    IQPT_THROW_FAILED(iqpt_rays_traced(m_ctx, &r));
    return r;
}

void path_tracer::read_linear(std::vector<float>& rgba) const {
    if (m_comm) {                 // collective: the whole frame's accumulator on rank 0
        rgba.resize((size_t)m_camera->get_width() * m_camera->get_height() * 4);
        IQPT_THROW_FAILED(iqpt_gather_read_select(m_ctx, 0, IQPT_GATHER_ACCUM, rgba.data(), nullptr));
        return;
    }
    uint64_t n = 0;
    IQPT_THROW_FAILED(iqpt_num_pixels(m_ctx, &n));
    rgba.resize((size_t)n * 4);
    IQPT_THROW_FAILED(iqpt_read(m_ctx, rgba.data(), nullptr));
}

void path_tracer::save_checkpoint(const std::string& path) const {
    IQPT_THROW_FAILED(iqpt_checkpoint_save(m_ctx, path.c_str()));
}

void path_tracer::load_checkpoint(const std::string& path) {
    IQPT_THROW_FAILED(iqpt_checkpoint_load(m_ctx, path.c_str()));
    m_pending_reset = false;       // the loaded state replaces any reset not yet applied
}

}  // namespace iqpt
