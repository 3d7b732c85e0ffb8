// rt_hip_binding.cpp -- the reference-side binding: what a maintainer of
// zachoines/simple-raytracer adds to route its hot path through this repo's
// C ABI (include/rt_hip.h, librt_hip.so).
//
// It defines the reference's own seam,
//
//     Mat3D create_view_window_and_ray_trace(Vector3 view_origin,
//         Vector3 view_direction, Vector3 view_up, float fov_h, float res_h,
//         float res_w, Color background_color);          // main.cpp:12-20, :670
//
// with the reference's types (src/definitions.h, read in place with
// -I<reference>), so the call at main.cpp:607 reaches the GPU path once this
// file replaces the reference's definition (main.cpp:670-767).  It reads the
// scene from the reference's global `Globals environment` (main.cpp:58,
// src/definitions.h:304-311) exactly as TraceRay / ShadeRay do, hands it over
// as an rt_scene_desc, renders, and quantises into the reference's Mat3D.
//
// Built two ways (no reference source is copied into this repo):
//   * tests/test_integration.py: g++ -std=c++20 -fsyntax-only -I<reference>
//     -Iinclude integration/rt_hip_binding.cpp;
//   * oracle/Makefile `ref-hip`: linked with the reference's own main.cpp
//     (its definition of the seam made weak) into oracle/_ref/SimpleRayTracer_hip
//     -- the reference's parser and writer with this repo's hot path; a GPU test
//     compares its PPMs with the reference's.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

// src/config.h defines the keyword table `argsStringValues` (a global
// std::map) in the header itself; the reference's main.cpp owns that
// definition, so this translation unit gives its copy another name.
#define argsStringValues rt_binding_unused_keyword_table
#include "src/definitions.h"
#undef argsStringValues

#include "rt_hip.h"
#include "rt_host.h"

extern Globals environment;   // main.cpp:58

namespace {

rt_material to_material(const Material &m) {                         // src/definitions.h:249-254
    rt_material r;
    r.diffuse[0] = m.diffuse.r, r.diffuse[1] = m.diffuse.g, r.diffuse[2] = m.diffuse.b;
    r.specular[0] = m.specular.r, r.specular[1] = m.specular.g, r.specular[2] = m.specular.b;
    r.ka = m.ka, r.kd = m.kd, r.ks = m.ks, r.n = m.n;
    r.opacity = m.opacity;
    r.eta = m.refraction_index;
    return r;
}

// The textures the objects use, each once: Texture::image is a Mat3D indexed
// (x, y, channel) with values 0..255 (src/utility.h:123-130); the ABI takes
// rows of RGB bytes, [y][x][3].
struct TextureTable {
    std::map<const Texture *, int> index;
    std::vector<std::vector<unsigned char>> bytes;
    std::vector<rt_texture_desc> descs;

    int id_of(const SceneObjectInfo *o) {
        if (!o->has_texture || !o->texture) return -1;
        auto it = index.find(o->texture);
        if (it != index.end()) return it->second;
        Texture *t = o->texture;
        const int w = (int)t->width, h = (int)t->height;
        std::vector<unsigned char> px((size_t)w * h * 3);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++)
                for (int c = 0; c < 3; c++) px[((size_t)y * w + x) * 3 + c] = (unsigned char)t->image->get(x, y, c);
        bytes.push_back(std::move(px));
        const int id = (int)descs.size();
        descs.push_back(rt_texture_desc{w, h, nullptr});
        index[o->texture] = id;
        return id;
    }
    void finish() {   // the byte vectors no longer move: point the descriptors at them
        for (size_t k = 0; k < descs.size(); k++) descs[k].rgb = bytes[k].data();
    }
};

void put3(float out[3], Vector3 a) { out[0] = a.x, out[1] = a.y, out[2] = a.z; }

}  // namespace

Mat3D create_view_window_and_ray_trace(Vector3 view_origin, Vector3 view_direction, Vector3 view_up, float fov_h,
                                       float res_h, float res_w, Color background_color) {
    // --- the scene, in the order TraceRay visits it (main.cpp:1218: every
    // "face" before every "sphere", each type in file order)
    TextureTable tex;
    std::vector<rt_face_desc> faces;
    std::vector<rt_sphere_desc> spheres;
    for (SceneObjectInfo *o : environment.scene_object_infos["face"]) {
        const Face *fc = environment.faces[(int)o->id];
        rt_face_desc fd{};
        for (int k = 0; k < 3; k++) {
            fd.v[k][0] = fc->vertex[k].x, fd.v[k][1] = fc->vertex[k].y, fd.v[k][2] = fc->vertex[k].z;
            fd.vn[k][0] = fc->vertex_normal[k].x, fd.vn[k][1] = fc->vertex_normal[k].y;
            fd.vn[k][2] = fc->vertex_normal[k].z;
            fd.vt[k][0] = fc->texture_coords[k].x, fd.vt[k][1] = fc->texture_coords[k].y;
        }
        fd.smooth = fc->smooth_shading ? 1 : 0;
        fd.mat = to_material(o->material);
        fd.texture = tex.id_of(o);
        faces.push_back(fd);
    }
    for (SceneObjectInfo *o : environment.scene_object_infos["sphere"]) {
        const Sphere *sp = environment.spheres[(int)o->id];
        rt_sphere_desc sd{};
        sd.center[0] = sp->center.x, sd.center[1] = sp->center.y, sd.center[2] = sp->center.z;
        sd.radius = sp->radius;
        sd.mat = to_material(o->material);
        sd.texture = tex.id_of(o);
        spheres.push_back(sd);
    }
    tex.finish();
    std::vector<rt_light_desc> lights;                                  // main.cpp:378-411, file order
    for (const Light &lt : environment.scene_lights) {
        rt_light_desc ld{};
        put3(ld.xyz, lt.w == 0 ? lt.direction : lt.position);
        ld.w = lt.w;
        ld.color[0] = lt.color.r, ld.color[1] = lt.color.g, ld.color[2] = lt.color.b;
        lights.push_back(ld);
    }
    rt_scene_desc desc{};
    desc.n_spheres = (int)spheres.size();
    desc.spheres = spheres.data();
    desc.n_faces = (int)faces.size();
    desc.faces = faces.data();
    desc.n_lights = (int)lights.size();
    desc.lights = lights.data();
    desc.n_textures = (int)tex.descs.size();
    desc.textures = tex.descs.data();
    desc.bkg[0] = background_color.r, desc.bkg[1] = background_color.g, desc.bkg[2] = background_color.b;
    // main.cpp:751 reads it through std::map::operator[]: 0 unless bkgcolor had a 4th value
    desc.eta_bkg = environment.other["bkg_refraction_index"];
    desc.epsilon = environment.other["epsilon"];                        // main.cpp:101
    desc.depth = (int)environment.other["recursion_depth"];             // main.cpp:100

    // --- the view window, main.cpp:677-710, in the reference's own Vector3
    // arithmetic (d = 5.0 is src/config.h's view-plane distance, a double)
    Vector3 u_axis = view_direction.cross(view_up).norm();
    Vector3 v_axis = u_axis.cross(view_direction);
    float aspect = res_w / res_h;
    float win_w = 2.0f * d * tan((0.5 * fov_h) * M_PI / 180.0f);
    float win_h = win_w / aspect;
    Vector3 centre = view_origin + view_direction * d;
    Vector3 ul = centre - u_axis * (win_w / 2.0f) + v_axis * (win_h / 2.0f);
    Vector3 ur = centre + u_axis * (win_w / 2.0f) + v_axis * (win_h / 2.0f);
    Vector3 ll = centre - u_axis * (win_w / 2.0f) - v_axis * (win_h / 2.0f);
    rt_camera cam;
    put3(cam.eye, view_origin);
    put3(cam.ul, ul);
    put3(cam.dh, (ur - ul) / (res_w - 1.0f));
    put3(cam.dv, (ll - ul) / (res_h - 1.0f));

    // --- the pixel loop main.cpp:718-764 and everything under it, on the GPU
    const int W = (int)res_w, H = (int)res_h;
    std::vector<float> rgb((size_t)W * H * 3);
    rt_scene *scene = nullptr;
    rt_stats st{};
    int rc = rt_scene_create(0, &desc, &scene);
    // the kernel without counters unless RT_HIP_SEAM_STATS asks for the counts below
    const bool seam_stats = std::getenv("RT_HIP_SEAM_STATS") != nullptr;
    if (rc == RT_OK) rc = rt_scene_set_option(scene, "counters", seam_stats ? 1 : 0);
    if (rc == RT_OK) rc = rt_render_rows(scene, &cam, W, H, 0, H, rgb.data(), &st);
    rt_scene_destroy(scene);
    if (rc != RT_OK) throw std::runtime_error(std::string("rt_hip render failed: ") + rt_strerror(rc));
    // RT_HIP_SEAM_STATS set: say that this seam ran, with the GPU's TraceRay
    // counts (a test asserts them against the reference's own call counts)
    if (seam_stats)
        std::fprintf(stderr, "rt_hip seam: %dx%d rays primary %llu shadow %llu refraction %llu reflection %llu\n", W, H,
                     st.primary, st.shadow, st.refraction, st.reflection);

    // --- quantisation main.cpp:760-762 into the reference's image type
    std::vector<long long> q(rgb.size());
    rth_quantize(rgb.data(), (long long)q.size(), q.data());
    Mat3D matt(res_h, res_w, 3, 0);                                     // main.cpp:717
    for (int i = 0; i < H; i++)
        for (int j = 0; j < W; j++)
            for (int c = 0; c < 3; c++) matt(i, j, c) = (size_t)q[((size_t)i * W + j) * 3 + c];
    return matt;
}
