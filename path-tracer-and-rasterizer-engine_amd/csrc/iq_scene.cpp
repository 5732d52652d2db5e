// iq_scene.cpp — scene / mesh / model builders and the camera constructor (host only).
//
// Restates IoniqRE/mesh.cu (procedural meshes), IoniqRE/model.cu (model transform),
// IoniqRE/scene.cu:104-181 (build_packet: sorted-name mesh ids, drawcall arrays) and
// IoniqRE/camera.cu:5-18 (view/projection and inverses) behind the iqpt_scene_* / iqpt_camera_init
// C ABI. The D3D11 vertex/index buffers of mesh::setup_mesh (mesh.cu:37-64) are out of scope.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "iq_host_math.hpp"
#include "iqpt.h"
#include "iqpt_internal.hpp"

namespace {

using iq::mat4;
using iq::usage;
using iq::vec4;

struct mesh {
    std::vector<iqpt_vertex> vertices;
    std::vector<uint32_t> indices;
    int type = IQPT_MESH_TRIANGLES;
};

iqpt_vertex make_vertex(const vec4& p, const vec4& n) {
    iqpt_vertex v;
    v.pos[0] = p.x; v.pos[1] = p.y; v.pos[2] = p.z;
    v.normal[0] = n.x; v.normal[1] = n.y; v.normal[2] = n.z;
    return v;
}

mesh make_tri() {                                                               // mesh.cu:66-80
    mesh m;
    const vec4 n(0.0f, 0.0f, -1.0f, 0.0f);
    m.vertices = {make_vertex({0.0f, 0.5f, 0.0f, 0.0f}, n), make_vertex({0.5f, -0.5f, 0.0f, 0.0f}, n),
                  make_vertex({-0.5f, -0.5f, 0.0f, 0.0f}, n)};
    m.indices = {0, 1, 2};
    return m;
}

mesh make_quad() {                                                              // mesh.cu:82-98
    mesh m;
    const vec4 n(0.0f, 0.0f, -1.0f, 0.0f);
    m.vertices = {make_vertex({-0.5f, -0.5f, 0.0f, 0.0f}, n), make_vertex({0.5f, -0.5f, 0.0f, 0.0f}, n),
                  make_vertex({0.5f, 0.5f, 0.0f, 0.0f}, n), make_vertex({-0.5f, 0.5f, 0.0f, 0.0f}, n)};
    m.indices = {0, 3, 1, 1, 3, 2};
    return m;
}

mesh make_reg_polygon(uint32_t vertices) {                                     // mesh.cu:100-128
    mesh m;
    vertices = vertices > 2 ? vertices : 3;
    const float theta = IQ_TAU / (float)vertices;
    const vec4 n(0.0f, 0.0f, -1.0f, 0.0f);
    m.vertices.push_back(make_vertex(vec4(), n));
    vec4 v(0.5f, 0.0f, 0.0f, 0.0f);
    m.vertices.push_back(make_vertex(v, n));
    const mat4 tr = iq::rotation_z(theta);
    for (uint32_t i = 1; i < vertices; i++) {
        v = iq::transformed(v, tr, usage::POINT);
        m.vertices.push_back(make_vertex(v, n));
    }
    for (uint32_t i = 1; i < vertices; i++) {
        m.indices.push_back(i);
        m.indices.push_back(0);
        m.indices.push_back(i + 1);
    }
    m.indices.push_back((uint32_t)m.vertices.size() - 1);
    m.indices.push_back(0);
    m.indices.push_back(1);
    return m;
}

mesh make_cube() {                                                              // mesh.cu:130-186
    mesh m;
    struct R { float p[3]; float n[3]; };
    static const R rows[24] = {
        {{-0.5f, -0.5f, -0.5f}, {0, 0, -1}}, {{0.5f, -0.5f, -0.5f}, {0, 0, -1}},
        {{0.5f, 0.5f, -0.5f}, {0, 0, -1}},   {{-0.5f, 0.5f, -0.5f}, {0, 0, -1}},
        {{-0.5f, -0.5f, 0.5f}, {0, 0, 1}},   {{0.5f, -0.5f, 0.5f}, {0, 0, 1}},
        {{0.5f, 0.5f, 0.5f}, {0, 0, 1}},     {{-0.5f, 0.5f, 0.5f}, {0, 0, 1}},
        {{-0.5f, -0.5f, 0.5f}, {-1, 0, 0}},  {{-0.5f, 0.5f, -0.5f}, {-1, 0, 0}},
        {{-0.5f, -0.5f, -0.5f}, {-1, 0, 0}}, {{-0.5f, 0.5f, 0.5f}, {-1, 0, 0}},
        {{0.5f, -0.5f, -0.5f}, {1, 0, 0}},   {{0.5f, 0.5f, 0.5f}, {1, 0, 0}},
        {{0.5f, -0.5f, 0.5f}, {1, 0, 0}},    {{0.5f, 0.5f, -0.5f}, {1, 0, 0}},
        {{-0.5f, -0.5f, 0.5f}, {0, -1, 0}},  {{0.5f, -0.5f, -0.5f}, {0, -1, 0}},
        {{0.5f, -0.5f, 0.5f}, {0, -1, 0}},   {{-0.5f, -0.5f, -0.5f}, {0, -1, 0}},
        {{-0.5f, 0.5f, -0.5f}, {0, 1, 0}},   {{0.5f, 0.5f, 0.5f}, {0, 1, 0}},
        {{0.5f, 0.5f, -0.5f}, {0, 1, 0}},    {{-0.5f, 0.5f, 0.5f}, {0, 1, 0}},
    };
    for (const R& r : rows) {
        iqpt_vertex v;
        std::memcpy(v.pos, r.p, sizeof v.pos);
        std::memcpy(v.normal, r.n, sizeof v.normal);
        m.vertices.push_back(v);
    }
    m.indices = {0, 2, 1, 0, 3, 2, 5, 7, 4, 5, 6, 7, 8, 9, 10, 8, 11, 9,
                 12, 13, 14, 12, 15, 13, 16, 17, 18, 16, 19, 17, 20, 21, 22, 20, 23, 21};
    return m;
}

mesh make_uv_sphere(bool /*flat*/, uint32_t segments, uint32_t rings, int type) {  // mesh.cu:190-279
    mesh m;
    m.type = type;
    segments = segments > 2 ? segments : 3;
    rings = rings > 2 ? rings : 3;
    const float theta = IQ_PI / (float)rings;
    const float phi = IQ_TAU / (float)segments;
    const vec4 bottom(0.0f, -1.0f, 0.0f, 1.0f);
    const vec4 top(0.0f, 1.0f, 0.0f, 1.0f);
    const mat4 polar_tr = iq::rotation_z(theta);
    const mat4 azimuthal_tr = iq::rotation_y(phi);
    vec4 crt_polar = bottom;
    for (uint32_t i = 1; i < rings; i++) {
        crt_polar = iq::transformed(crt_polar, polar_tr, usage::POINT);
        m.vertices.push_back(make_vertex(crt_polar, crt_polar));
        vec4 crt_az = crt_polar;
        for (uint32_t j = 1; j < segments; j++) {
            crt_az = iq::transformed(crt_az, azimuthal_tr, usage::POINT);
            m.vertices.push_back(make_vertex(crt_az, crt_az));
        }
    }
    m.vertices.push_back(make_vertex(bottom, bottom));
    m.vertices.push_back(make_vertex(top, top));
    for (uint32_t i = 0; i < rings - 2; i++) {
        for (uint32_t j = 0; j < segments - 1; j++) {
            m.indices.push_back(i * segments + j);
            m.indices.push_back(i * segments + j + 1);
            m.indices.push_back((i + 1) * segments + j + 1);
            m.indices.push_back(i * segments + j);
            m.indices.push_back((i + 1) * segments + j + 1);
            m.indices.push_back((i + 1) * segments + j);
        }
        m.indices.push_back((i + 1) * segments - 1);
        m.indices.push_back(i * segments);
        m.indices.push_back((i + 1) * segments);
        m.indices.push_back((i + 1) * segments - 1);
        m.indices.push_back((i + 1) * segments);
        m.indices.push_back((i + 2) * segments - 1);
    }
    const uint32_t top_idx = (uint32_t)m.vertices.size() - 1;
    const uint32_t bottom_idx = top_idx - 1;
    const uint32_t nv = (uint32_t)m.vertices.size();
    for (uint32_t i = 0; i < segments - 1; i++) {
        m.indices.push_back(bottom_idx);
        m.indices.push_back(i + 1);
        m.indices.push_back(i);
        m.indices.push_back(top_idx);
        m.indices.push_back(nv - i - 4);
        m.indices.push_back(nv - i - 3);
    }
    m.indices.push_back(bottom_idx);
    m.indices.push_back(0);
    m.indices.push_back(segments - 1);
    m.indices.push_back(top_idx);
    m.indices.push_back(nv - 3);
    m.indices.push_back(nv - segments - 2);
    return m;
}

struct model {
    std::string mesh_name;
    vec4 scale_v{1.0f}, rotation{0.0f}, translation{0.0f};
    mat4 transform;
    uint64_t order = 0;                         // insertion order: tie-break of scene.h:58-67
    int64_t material = -1;                      // material table index (-1: the reference default)
    void recompute() {                                                          // model.cu:11-18
        mat4 s = iq::scale(scale_v);
        mat4 r = iq::rotation_x(rotation.x) * iq::rotation_y(rotation.y) * iq::rotation_z(rotation.z);
        mat4 t = iq::translate(translation);
        transform = s * r * t;
    }
};

}  // namespace

struct iqpt_scene {
    std::map<std::string, mesh> meshes;
    std::map<std::string, model> models;
    uint64_t next_order = 0;
    std::vector<iqpt_material> materials;      // §8f.3 material table (empty: reference materials)
    // storage of the last built packet
    std::vector<iqpt_tri_mesh> pk_meshes;
    std::vector<iqpt_tri_mesh_drawcall> pk_tri_dcs;
    std::vector<iqpt_sphere_drawcall> pk_sph_dcs;
    std::vector<iqpt_material> pk_mats;
    std::vector<uint32_t> pk_tri_mat, pk_sph_mat;
};

namespace {
int add_mesh(iqpt_scene* s, const char* name, mesh&& m) {
    if (!s || !name) return iqpt::fail(IQPT_ERR_INVALID_ARG, "scene/name is NULL");
    s->meshes.emplace(name, std::move(m));      // scene.cu:9-15: an existing name is kept
    return IQPT_OK;
}
}  // namespace

extern "C" {

int iqpt_scene_create(iqpt_scene** out) {
    if (!out) return iqpt::fail(IQPT_ERR_INVALID_ARG, "out is NULL");
    *out = new iqpt_scene();
    return IQPT_OK;
}

int iqpt_scene_destroy(iqpt_scene* s) {
    delete s;
    return IQPT_OK;
}

int iqpt_scene_add_mesh_tri(iqpt_scene* s, const char* name) { return add_mesh(s, name, make_tri()); }
int iqpt_scene_add_mesh_quad(iqpt_scene* s, const char* name) { return add_mesh(s, name, make_quad()); }
int iqpt_scene_add_mesh_reg_polygon(iqpt_scene* s, const char* name, uint32_t vertices) {
    return add_mesh(s, name, make_reg_polygon(vertices));
}
int iqpt_scene_add_mesh_cube(iqpt_scene* s, const char* name) { return add_mesh(s, name, make_cube()); }
int iqpt_scene_add_mesh_uv_sphere(iqpt_scene* s, const char* name, int flat, uint32_t segments,
                                  uint32_t rings, int mesh_type) {
    if (mesh_type != IQPT_MESH_TRIANGLES && mesh_type != IQPT_MESH_SPHERES)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "mesh_type must be IQPT_MESH_TRIANGLES or IQPT_MESH_SPHERES");
    return add_mesh(s, name, make_uv_sphere(flat != 0, segments, rings, mesh_type));
}
int iqpt_scene_add_mesh(iqpt_scene* s, const char* name, int mesh_type, const iqpt_vertex* vertices,
                        uint32_t num_vertices, const uint32_t* indices, uint32_t num_indices) {
    if (mesh_type != IQPT_MESH_TRIANGLES && mesh_type != IQPT_MESH_SPHERES)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "bad mesh_type");
    if ((num_vertices && !vertices) || (num_indices && !indices))
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL vertex/index array");
    mesh m;
    m.type = mesh_type;
    m.vertices.assign(vertices, vertices + num_vertices);
    m.indices.assign(indices, indices + num_indices);
    return add_mesh(s, name, std::move(m));
}

int iqpt_scene_add_model(iqpt_scene* s, const char* name, const char* mesh_name, const float scale[4],
                         const float rotation[4], const float translation[4]) {
    if (!s || !name || !mesh_name) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (s->models.count(name)) return IQPT_OK;   // scene.cu:47-52: insertion does not take place
    model m;
    m.mesh_name = mesh_name;
    if (scale) m.scale_v = vec4(scale[0], scale[1], scale[2], scale[3]);
    if (rotation) m.rotation = vec4(rotation[0], rotation[1], rotation[2], rotation[3]);
    if (translation) m.translation = vec4(translation[0], translation[1], translation[2], translation[3]);
    m.recompute();
    m.order = s->next_order++;
    // scene.cu:56: m_meshes[mesh_name] default-constructs a missing mesh (empty, TRIANGLES)
    s->meshes[mesh_name];
    s->models.emplace(name, m);
    return IQPT_OK;
}

int iqpt_scene_add_material(iqpt_scene* s, const iqpt_material* m, uint32_t* index) {
    if (!s || !m) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    if (m->type != IQPT_MAT_EMISSIVE && m->type != IQPT_MAT_OREN_NAYAR)
        return iqpt::fail(IQPT_ERR_INVALID_ARG, "unknown material type");
    if (s->materials.size() >= 0xffff) return iqpt::fail(IQPT_ERR_INVALID_ARG, "too many materials");
    s->materials.push_back(*m);
    if (index) *index = (uint32_t)(s->materials.size() - 1);
    return IQPT_OK;
}

int iqpt_scene_set_model_material(iqpt_scene* s, const char* model_name, uint32_t material) {
    if (!s || !model_name) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    auto it = s->models.find(model_name);
    if (it == s->models.end()) return iqpt::fail(IQPT_ERR_INVALID_ARG, std::string("no model ") + model_name);
    if (material >= s->materials.size()) return iqpt::fail(IQPT_ERR_INVALID_ARG, "material index out of range");
    it->second.material = material;
    return IQPT_OK;
}

int iqpt_scene_num_meshes(const iqpt_scene* s, uint32_t* n) {
    if (!s || !n) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    *n = (uint32_t)s->meshes.size();
    return IQPT_OK;
}

int iqpt_scene_build_packet(iqpt_scene* s, iqpt_packet_desc* out) {            // scene.cu:104-181
    if (!s || !out) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    std::vector<std::string> names;
    for (const auto& kv : s->meshes) names.push_back(kv.first);

    s->pk_meshes.clear();
    s->pk_tri_dcs.clear();
    s->pk_sph_dcs.clear();
    s->pk_tri_mat.clear();
    s->pk_sph_mat.clear();
    // the table, followed by the reference's two materials for models without an assignment
    // (path_tracer.cu:248-249: oren_nayar(iqvec(.5,.5,.5,0), 1), emissive(iqvec(1), 10))
    const bool with_table = !s->materials.empty();
    s->pk_mats = s->materials;
    const uint32_t def_emissive = (uint32_t)s->pk_mats.size();
    const uint32_t def_oren_nayar = def_emissive + 1;
    if (with_table) {
        s->pk_mats.push_back(iqpt_material{IQPT_MAT_EMISSIVE, {1.0f, 1.0f, 1.0f, 1.0f}, 10.0f});
        s->pk_mats.push_back(iqpt_material{IQPT_MAT_OREN_NAYAR, {0.5f, 0.5f, 0.5f, 0.0f}, 1.0f});
    }
    for (const auto& n : names) {
        const mesh& m = s->meshes.at(n);
        if (m.type != IQPT_MESH_TRIANGLES) continue;
        iqpt_tri_mesh tm;
        tm.vertices = m.vertices.data();
        tm.indices = m.indices.data();
        tm.num_indices = (uint32_t)m.indices.size();
        tm.num_vertices = (uint32_t)m.vertices.size();
        s->pk_meshes.push_back(tm);
    }
    // models sorted by (mesh name, insertion order) — scene.h:58-67
    std::vector<const model*> sorted;
    for (const auto& kv : s->models) sorted.push_back(&kv.second);
    std::sort(sorted.begin(), sorted.end(), [](const model* a, const model* b) {
        if (a->mesh_name != b->mesh_name) return a->mesh_name < b->mesh_name;
        return a->order < b->order;
    });
    uint32_t mesh_id = UINT32_MAX;
    std::string last;
    bool first = true;
    for (const model* pm : sorted) {
        if (first || pm->mesh_name != last) {
            first = false;
            last = pm->mesh_name;
            // lower_bound over ALL names from mesh_id + 1 (wraps to 0), scene.cu:167
            mesh_id = (uint32_t)(std::lower_bound(names.begin() + (uint32_t)(mesh_id + 1u), names.end(), last) -
                                 names.begin());
        }
        const mesh& m = s->meshes.at(last);
        if (m.type == IQPT_MESH_TRIANGLES) {
            iqpt_tri_mesh_drawcall dc;
            std::memcpy(dc.transform, pm->transform.m, sizeof dc.transform);
            dc.mesh_id = mesh_id;
            s->pk_tri_dcs.push_back(dc);
            s->pk_tri_mat.push_back(pm->material >= 0 ? (uint32_t)pm->material : def_emissive);
        } else {
            iqpt_sphere_drawcall dc;
            dc.center[0] = pm->translation.x; dc.center[1] = pm->translation.y;
            dc.center[2] = pm->translation.z; dc.center[3] = pm->translation.w;
            dc.radius = pm->scale_v.x;
            s->pk_sph_dcs.push_back(dc);
            s->pk_sph_mat.push_back(pm->material >= 0 ? (uint32_t)pm->material : def_oren_nayar);
        }
    }
    out->num_drawcalls[IQPT_MESH_TRIANGLES] = (uint32_t)s->pk_tri_dcs.size();
    out->num_drawcalls[IQPT_MESH_SPHERES] = (uint32_t)s->pk_sph_dcs.size();
    out->num_tri_meshes = (uint32_t)s->pk_meshes.size();
    out->tri_meshes = s->pk_meshes.empty() ? nullptr : s->pk_meshes.data();
    out->tri_mesh_dcs = s->pk_tri_dcs.empty() ? nullptr : s->pk_tri_dcs.data();
    out->sphere_dcs = s->pk_sph_dcs.empty() ? nullptr : s->pk_sph_dcs.data();
    out->materials = with_table ? s->pk_mats.data() : nullptr;
    out->num_materials = with_table ? (uint32_t)s->pk_mats.size() : 0u;
    out->tri_dc_material = with_table && !s->pk_tri_mat.empty() ? s->pk_tri_mat.data() : nullptr;
    out->sphere_dc_material = with_table && !s->pk_sph_mat.empty() ? s->pk_sph_mat.data() : nullptr;
    return IQPT_OK;
}

int iqpt_scene_add_preset(iqpt_scene* s, const char* preset) {
    if (!s || !preset) return iqpt::fail(IQPT_ERR_INVALID_ARG, "NULL argument");
    const std::string name(preset);
    auto add = [&](const char* model_name, const char* mesh_name, vec4 sc, vec4 rot, vec4 tr) {
        const float a[4] = {sc.x, sc.y, sc.z, sc.w}, b[4] = {rot.x, rot.y, rot.z, rot.w},
                    c[4] = {tr.x, tr.y, tr.z, tr.w};
        return iqpt_scene_add_model(s, model_name, mesh_name, a, b, c);
    };
    const vec4 zero(0.0f);
    if (name == "app_default") {                                   // application.cu:25-34
        iqpt_scene_add_mesh_tri(s, "default");
        iqpt_scene_add_mesh_cube(s, "cube");
        iqpt_scene_add_mesh_uv_sphere(s, "sphere", 0, 128, 64, IQPT_MESH_SPHERES);
        add("ground", "sphere", vec4(10.0f), vec4(IQ_PI_DIV_2, 0.0f, 0.0f, 0.0f), vec4(0.0f, -10.0f, 0.0f, 0.0f));
        add("sph", "sphere", vec4(0.5f), zero, vec4(0.0f, 0.5f, 0.0f, 0.0f));
        add("wall", "cube", vec4(1.0f), zero, vec4(1.0f, 0.5f, 0.0f, 0.0f));
        return IQPT_OK;
    }
    if (name == "c1_plumbing") {
        iqpt_scene_add_mesh_uv_sphere(s, "light", 0, 16, 8, IQPT_MESH_TRIANGLES);
        iqpt_scene_add_mesh_uv_sphere(s, "sphere", 0, 32, 16, IQPT_MESH_SPHERES);
        add("lamp", "light", vec4(0.5f), zero, vec4(1.0f, 1.0f, 0.0f, 0.0f));
        add("ball", "sphere", vec4(0.5f), zero, vec4(0.0f, 0.5f, 0.0f, 0.0f));
        return IQPT_OK;
    }
    if (name == "cornell") {
        iqpt_scene_add_mesh_quad(s, "quad");
        iqpt_scene_add_mesh_uv_sphere(s, "sphere", 0, 32, 16, IQPT_MESH_SPHERES);
        const vec4 wall(2.0f, 2.0f, 1.0f, 1.0f);
        add("back", "quad", wall, zero, vec4(0.0f, 0.5f, 1.0f, 0.0f));
        add("floor", "quad", wall, vec4(IQ_PI_DIV_2, 0.0f, 0.0f, 0.0f), vec4(0.0f, -0.5f, 0.0f, 0.0f));
        add("ceiling", "quad", wall, vec4(-IQ_PI_DIV_2, 0.0f, 0.0f, 0.0f), vec4(0.0f, 1.5f, 0.0f, 0.0f));
        add("left", "quad", wall, vec4(0.0f, IQ_PI_DIV_2, 0.0f, 0.0f), vec4(-1.0f, 0.5f, 0.0f, 0.0f));
        add("right", "quad", wall, vec4(0.0f, -IQ_PI_DIV_2, 0.0f, 0.0f), vec4(1.0f, 0.5f, 0.0f, 0.0f));
        add("sphere_big", "sphere", vec4(0.35f), zero, vec4(-0.4f, -0.15f, 0.2f, 0.0f));
        add("sphere_small", "sphere", vec4(0.25f), zero, vec4(0.45f, -0.25f, -0.2f, 0.0f));
        return IQPT_OK;
    }
    if (name == "cornell_lit") {
        // §8f.3: the C2 geometry with a material table — Oren–Nayar walls (white, red, green), a small
        // emissive ceiling panel, diffuse spheres — a lit Cornell box instead of the reference's
        // all-emissive walls
        iqpt_scene_add_mesh_quad(s, "quad");
        iqpt_scene_add_mesh_uv_sphere(s, "sphere", 0, 32, 16, IQPT_MESH_SPHERES);
        const vec4 wall(2.0f, 2.0f, 1.0f, 1.0f);
        add("back", "quad", wall, zero, vec4(0.0f, 0.5f, 1.0f, 0.0f));
        add("floor", "quad", wall, vec4(IQ_PI_DIV_2, 0.0f, 0.0f, 0.0f), vec4(0.0f, -0.5f, 0.0f, 0.0f));
        add("ceiling", "quad", wall, vec4(-IQ_PI_DIV_2, 0.0f, 0.0f, 0.0f), vec4(0.0f, 1.5f, 0.0f, 0.0f));
        add("left", "quad", wall, vec4(0.0f, IQ_PI_DIV_2, 0.0f, 0.0f), vec4(-1.0f, 0.5f, 0.0f, 0.0f));
        add("right", "quad", wall, vec4(0.0f, -IQ_PI_DIV_2, 0.0f, 0.0f), vec4(1.0f, 0.5f, 0.0f, 0.0f));
        add("light", "quad", vec4(0.6f, 0.6f, 1.0f, 1.0f), vec4(-IQ_PI_DIV_2, 0.0f, 0.0f, 0.0f),
            vec4(0.0f, 1.49f, 0.0f, 0.0f));
        add("sphere_big", "sphere", vec4(0.35f), zero, vec4(-0.4f, -0.15f, 0.2f, 0.0f));
        add("sphere_small", "sphere", vec4(0.25f), zero, vec4(0.45f, -0.25f, -0.2f, 0.0f));
        const iqpt_material mats[] = {
            {IQPT_MAT_OREN_NAYAR, {0.73f, 0.73f, 0.73f, 0.0f}, 0.5f},   // 0 white walls
            {IQPT_MAT_OREN_NAYAR, {0.65f, 0.05f, 0.05f, 0.0f}, 0.5f},   // 1 red
            {IQPT_MAT_OREN_NAYAR, {0.12f, 0.45f, 0.15f, 0.0f}, 0.5f},   // 2 green
            {IQPT_MAT_EMISSIVE, {1.0f, 0.9f, 0.75f, 1.0f}, 12.0f},      // 3 light
            {IQPT_MAT_OREN_NAYAR, {0.8f, 0.8f, 0.8f, 0.0f}, 0.2f},      // 4 big sphere
            {IQPT_MAT_OREN_NAYAR, {0.9f, 0.6f, 0.2f, 0.0f}, 1.0f},      // 5 small sphere
        };
        for (const iqpt_material& m : mats) iqpt_scene_add_material(s, &m, nullptr);
        const char* assign[][2] = {{"back", "0"}, {"floor", "0"}, {"ceiling", "0"}, {"left", "1"}, {"right", "2"},
                                   {"light", "3"}, {"sphere_big", "4"}, {"sphere_small", "5"}};
        for (const auto& a : assign) iqpt_scene_set_model_material(s, a[0], (uint32_t)(a[1][0] - '0'));
        return IQPT_OK;
    }
    if (name == "mesh10k") {
        iqpt_scene_add_mesh_uv_sphere(s, "ball", 0, 100, 51, IQPT_MESH_TRIANGLES);
        add("ball", "ball", vec4(0.75f), zero, vec4(0.0f, 0.5f, 0.0f, 0.0f));
        return IQPT_OK;
    }
    if (name == "mixed") {
        iqpt_scene_add_mesh_uv_sphere(s, "ball", 0, 250, 101, IQPT_MESH_TRIANGLES);
        iqpt_scene_add_mesh_uv_sphere(s, "sphere", 0, 32, 16, IQPT_MESH_SPHERES);
        add("ball", "ball", vec4(0.6f), zero, vec4(0.0f, 0.6f, 0.5f, 0.0f));
        char nm[32];
        for (int i = 0; i < 999; ++i) {
            std::snprintf(nm, sizeof nm, "pebble%04d", i);
            add(nm, "sphere", vec4(0.04f), zero,
                vec4(-2.0f + 0.1f * (float)(i % 40), 0.04f, -0.5f + 0.1f * (float)(i / 40), 0.0f));
        }
        add("ground", "sphere", vec4(10.0f), zero, vec4(0.0f, -10.0f, 0.0f, 0.0f));
        return IQPT_OK;
    }
    return iqpt::fail(IQPT_ERR_INVALID_ARG, "unknown preset '" + name + "'");
}

int iqpt_camera_init(iqpt_camera* cam, uint16_t width, uint16_t height, float fovh_deg, float znear,
                     float zfar, const float position[4], const float forward[4]) {  // camera.cu:5-18
    if (!cam || width == 0 || height == 0) return iqpt::fail(IQPT_ERR_INVALID_ARG, "bad camera arguments");
    std::memset(cam, 0, sizeof *cam);
    cam->width = width;
    cam->height = height;
    cam->fovh = fovh_deg;
    const float def_pos[4] = {0.0f, 0.5f, -3.0f, 0.0f};                         // camera.h:26
    const float def_fwd[4] = {0.0f, -0.5f, 3.0f, 0.0f};                         // camera.h:27
    std::memcpy(cam->position, position ? position : def_pos, sizeof cam->position);
    std::memcpy(cam->forward, forward ? forward : def_fwd, sizeof cam->forward);
    const vec4 pos(cam->position[0], cam->position[1], cam->position[2], cam->position[3]);
    const vec4 fwd(cam->forward[0], cam->forward[1], cam->forward[2], cam->forward[3]);
    const mat4 view = iq::look_at(pos, pos + fwd);
    const mat4 proj = iq::perspective((float)width / (float)height, iq::to_radians(fovh_deg), znear, zfar);
    const mat4 inv_view = iq::inversed(view);
    const mat4 inv_proj = iq::inversed(proj);
    std::memcpy(cam->view, view.m, 64);
    std::memcpy(cam->projection, proj.m, 64);
    std::memcpy(cam->inv_view, inv_view.m, 64);
    std::memcpy(cam->inv_proj, inv_proj.m, 64);
    return IQPT_OK;
}

}  // extern "C"
