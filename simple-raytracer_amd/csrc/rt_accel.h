// rt_accel.h -- host side of the scene store and its acceleration structure,
// with no device call: what rt_scene_create derives from the scene
// description (the per-object arrays of DESIGN.md §2, the BVH sources), and
// the build of the device's trees (the main BVH plus one shadow-cone tree per
// directional light, rt_bvh.h).  rt_scene.cpp uploads the results; the build
// is timed and checked on the CPU by tools/bvh_bench.cpp
// (tests/test_bvh_host.py) without a GPU.
//
// Replaces the reference's per-ray object scans (TraceRay, main.cpp:1218-1403)
// by trees that only decide which primitives a ray is tested against; every
// test keeps the reference's arithmetic (rt_kernels.hip).
#pragma once

#include <cstdint>
#include <vector>

#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_hip.h"

namespace rt {

// BVH source of one object (the boxes' padding depends on the eye, so the
// tree is built per camera range, build_accel)
struct PrimSrc {
    int key;                           // object index: faces, then spheres (main.cpp:1218)
    bool sphere;
    float lo[3], hi[3];                // face: vertex bounds; sphere: centre +- r
    float c[3], r;                     // sphere centre / radius
    double cond;                       // face: |e1|^2 |e2|^2 / det
    float v[3][3];                     // face: its vertices (AccelOpts::presplit clips the triangle)
};

// Everything the device scene store holds, built on the host from the scene
// description (rt_scene_create), plus the BVH sources.
struct AccelInput {
    int nf = 0, ns = 0;
    float eps = 1e-3f;
    std::vector<float4> fscan;         // faces, 5 words each (rt_device.h)
    std::vector<float4> sscan;         // spheres (centre, r)
    std::vector<float> ofac;           // (float)(1 - opacity) per object (main.cpp:909)
    std::vector<ObjK> objs;
    std::vector<FaceShadeK> fsh;
    std::vector<LightK> lights;
    std::vector<PrimSrc> prims;
    float scene_lo[3] = {0, 0, 0}, scene_hi[3] = {0, 0, 0};
    bool secondary = false;            // some material reflects or refracts
    bool nan_fac = false;              // some shadow factor is NaN (no opaque early exit)
    double crossings = 0.0;            // objects a line across the scene meets on average
};

// rt_scene_desc -> the host arrays (exact per-face invariants, main.cpp:1280-1301)
void accel_input(const rt_scene_desc *desc, AccelInput &in);

// Bound D on the distance from any ray origin (the eye, or a point inside the
// scene's bounds) to any primitive: the BVH padding's scale.
double distance_bound(const AccelInput &in, const float eye[3]);

#ifndef RT_PRESPLIT_GAIN
#define RT_PRESPLIT_GAIN 0.9
#endif
constexpr double kPresplitGain = RT_PRESPLIT_GAIN;   // a piece is split when its halves' boxes have <= this of its area
struct AccelOpts {
    int bvh_leaf = 8;                  // leaf size limit of the collapse
    int collapse = 1;                  // binary -> 4-wide: 0 greedy, 1 SAH-optimal
    int node_milli = 500;              // SAH collapse: node visit cost, x1000 of a sphere test
    int threads = 0;                   // host threads for the build (0: automatic, 1: serial)
    int presplit = 0;                  // references per face at most (0/1: one; build_accel's presplit)
};

// The device's trees, ready to upload.
struct AccelTree {
    bool ok = false;                   // false: geometry the BVH cannot bound (the scan is used)
    std::vector<rtbvh::NodeDev> nodes;  // main tree first, then the cone trees; links are byte offsets
    std::vector<float4> rec;           // leaf records (rt_bvh.h leaf_records), padded by 3 words
    std::vector<int32_t> objleaf;      // per object: its leaf's link in the main tree
    std::vector<DirK> dirk;            // per light (directional lights only)
    int dir_mode = 0;                  // Params::dir_bf
    int depth = 0, max_stack = 0;      // main tree
    int stack_all = 0;                 // deepest worst-case stack over all trees
    long long main_nodes = 0;
    long long refs = 0;                // primitive references in the main tree (> objects with presplit)
    int presplit = 0;                  // references per face at most, as built
    double sah = 0.0;                  // the main tree's SAH cost (node visits + primitive tests per ray, rt_accel.cpp)
    int threads = 1;                   // host threads used
    // host time per phase (ms): primitive boxes, binary SAH build, collapse +
    // BFS order, leaf records, quantisation, cone trees
    double ms[6] = {0, 0, 0, 0, 0, 0};
};

// Build every tree for distance bound D (boxes padded, rt_bvh.h):
//   face   pad = 2^-16 * D * max(1, cond)                 (32x the rounding bound)
//   sphere radius' = sqrt(r^2 + 2^-18 D^2) + 2^-16 D     (discriminant error)
void build_accel(const AccelInput &in, double D, const AccelOpts &o, AccelTree &out);

// Host threads the build uses when AccelOpts::threads is 0: the process's CPU
// affinity, capped by OMP_NUM_THREADS when set, and by 16.
int accel_threads();

}  // namespace rt
