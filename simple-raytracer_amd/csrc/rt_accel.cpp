// rt_accel.cpp -- host side of the scene store and the BVH build (rt_accel.h).
#include "rt_accel.h"

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace rt {

namespace {

V3 f3(const float *p) { return {p[0], p[1], p[2]}; }

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

// Binary SAH tree over P, collapsed into 4-wide nodes (collapse 0: greedy,
// largest child area first; 1: SAH-optimal) and renumbered breadth-first
// (the top levels first: cache locality of the hot nodes).
// SAH cost of a collapsed tree per ray that enters its root, in sphere tests:
// node_cost per node entered plus the leaves' primitive costs, each weighted
// by its box's surface area over the root's (a diagnostic: AccelTree::sah).
double sah_of(const rtbvh::Result4 &Q, const std::vector<float> &costs, double node_cost) {
    if (Q.nodes.empty()) return 0.0;
    auto child = [](const rtbvh::Node4 &n, int i) {
        rtbvh::Box b;
        for (int k = 0; k < 3; k++) b.lo[k] = n.lo[k][i], b.hi[k] = n.hi[k][i];
        return b;
    };
    rtbvh::Box root;
    for (int i = 0; i < 4; i++)
        if (Q.nodes[0].link[i] != rtbvh::kEmpty) root.grow(child(Q.nodes[0], i));
    const double a0 = root.area();
    if (!(a0 > 0.0) || !std::isfinite(a0)) return 0.0;
    double c = node_cost;
    for (const auto &n : Q.nodes)
        for (int i = 0; i < 4; i++) {
            const int32_t l = n.link[i];
            if (l == rtbvh::kEmpty) continue;
            const double a = child(n, i).area() / a0;
            if (l >= 0) {
                c += node_cost * a;
            } else {
                const int v = -l - 1, first = v >> 4, count = v & 15;
                double w = 0.0;
                for (int q = 0; q < count; q++) w += costs[(size_t)first + q];
                c += a * w;
            }
        }
    return c;
}

// Pre-splitting (AccelOpts::presplit, after Ernst and Greiner's early split
// clipping): a face whose box is much larger than the face -- a thin or
// slanted triangle -- becomes several references, each with the box of the
// part of the triangle inside one piece of its box (the largest piece split
// at the middle of its longest axis, the triangle clipped to each half in
// double), so that the tree's boxes overlap less.  Exact: every point of the
// triangle lies in some piece's box, each piece padded as the whole face is
// (build_accel), so a ray that meets the face enters a leaf holding it; a
// leaf tests a face once however many of its references it holds
// (leaf_records), and a ray visiting two leaves of one face meets the same
// candidate twice -- the same closest hit, and the same answer for an any-hit
// search when the face's shadow factor is 0 or 1 (x 0 twice is x 0, x 1 is
// exact).  Faces with any other factor (translucent: a duplicate would
// multiply twice) keep one reference.
struct ClipBox {
    double lo[3], hi[3];
    double area() const {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};
// the box of the triangle's part inside [blo, bhi] (false: none)
bool clip_box(const float v[3][3], const double blo[3], const double bhi[3], ClipBox &out) {
    double poly[12][3], tmp[12][3];
    int n = 3;
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) poly[i][k] = v[i][k];
    for (int ax = 0; ax < 3 && n > 0; ax++)
        for (int side = 0; side < 2 && n > 0; side++) {
            const double s = side == 0 ? blo[ax] : bhi[ax];
            auto inside = [&](const double *p) { return side == 0 ? p[ax] >= s : p[ax] <= s; };
            int m = 0;
            for (int i = 0; i < n; i++) {
                const double *a = poly[i], *b = poly[(i + 1) % n];
                const bool ia = inside(a), ib = inside(b);
                if (ia) {
                    for (int k = 0; k < 3; k++) tmp[m][k] = a[k];
                    m++;
                }
                if (ia != ib) {
                    const double t = (s - a[ax]) / (b[ax] - a[ax]);
                    for (int k = 0; k < 3; k++) tmp[m][k] = a[k] + t * (b[k] - a[k]);
                    tmp[m][ax] = s;
                    m++;
                }
            }
            n = m;
            for (int i = 0; i < n; i++)
                for (int k = 0; k < 3; k++) poly[i][k] = tmp[i][k];
        }
    if (n == 0) return false;
    for (int k = 0; k < 3; k++) out.lo[k] = INFINITY, out.hi[k] = -INFINITY;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 3; k++)
            out.lo[k] = std::min(out.lo[k], std::max(poly[i][k], blo[k])),
            out.hi[k] = std::max(out.hi[k], std::min(poly[i][k], bhi[k]));
    return true;
}
// a face's pieces (at most max_refs; one when splitting does not pay): the
// largest piece is split while its halves' boxes have at most kPresplitGain
// of its box's area (host SAH over C3 / C4 at 0.5 ... 0.9: 0.9 lowest)
void split_face(const float v[3][3], int max_refs, std::vector<ClipBox> &pieces) {
    pieces.clear();
    ClipBox whole;
    for (int k = 0; k < 3; k++) {
        whole.lo[k] = std::min((double)v[0][k], std::min((double)v[1][k], (double)v[2][k]));
        whole.hi[k] = std::max((double)v[0][k], std::max((double)v[1][k], (double)v[2][k]));
    }
    pieces.push_back(whole);
    std::vector<bool> done(1, false);
    while ((int)pieces.size() < max_refs) {
        int best = -1;
        for (int i = 0; i < (int)pieces.size(); i++)
            if (!done[i] && (best < 0 || pieces[i].area() > pieces[best].area())) best = i;
        if (best < 0) break;
        const ClipBox b = pieces[best];
        int ax = 0;
        for (int k = 1; k < 3; k++)
            if (b.hi[k] - b.lo[k] > b.hi[ax] - b.lo[ax]) ax = k;
        const double mid = 0.5 * (b.lo[ax] + b.hi[ax]);
        double llo[3], lhi[3], rlo[3], rhi[3];
        for (int k = 0; k < 3; k++) llo[k] = rlo[k] = b.lo[k], lhi[k] = rhi[k] = b.hi[k];
        lhi[ax] = mid;
        rlo[ax] = mid;
        ClipBox L, R;
        const bool hl = clip_box(v, llo, lhi, L), hr = clip_box(v, rlo, rhi, R);
        // split only where the two pieces' boxes cover clearly less than the
        // piece did (a compact piece stays whole)
        if (!hl || !hr || L.area() + R.area() > kPresplitGain * b.area()) {
            done[best] = true;
            continue;
        }
        pieces[best] = L;
        pieces.push_back(R);
        done.push_back(false);
    }
}

bool build_wide(const AccelOpts &o, int threads, std::vector<rtbvh::Prim> &P, rtbvh::Result &R, rtbvh::Result4 &Q,
                double *ms, double *sah = nullptr) {
    auto t0 = Clock::now();
    rtbvh::Builder B(P);
    B.max_leaf = o.collapse ? 1 : o.bvh_leaf;
    B.trav_cost = 0.5f;                // SAH node cost, in sphere tests (A/B over 0.25-2: 0.5 best, round 1)
    B.threads = threads;
    if (!B.build(R) || R.nodes.empty()) return false;
    if (ms) ms[1] += ms_since(t0);
    t0 = Clock::now();
    if (o.collapse)
        rtbvh::collapse_sah<4>(R, Q, o.bvh_leaf, (float)o.node_milli / 1000.0f);
    else
        rtbvh::collapse<4>(R, Q);
    rtbvh::bfs_order(Q);
    if (ms) ms[2] += ms_since(t0);
    if (sah) *sah = sah_of(Q, R.costs, (double)o.node_milli / 1000.0);
    return true;
}

// Shadow-cone tree of a directional light (Params::dirk, dir_bf == 2).
//
// The reference's directional shadow ray runs TraceRay with the light's
// UNNORMALISED direction d = -dir (main.cpp:895), and the sphere test
// assumes |d| = 1 (main.cpp:1225-1258).  With s = |d|, n = d / s, k = s^2 - 1,
// h = n.(c - o) (how far the centre is ahead of the origin along the ray) and
// l = the lateral distance of c from the ray's line, the discriminant is
//     det / 4 = (d.w)^2 - |w|^2 + r^2 = k h^2 - l^2 + r^2,
// and the sphere shadows o iff det >= 0 and its far root (-B + sqrt det) / 2
// exceeds epsilon: for h < 0 that needs o inside the sphere; for h >= 0 it is
// l^2 <= r^2 + k h^2 -- a cylinder (s = 1), a cone widening away from the
// light (s > 1) or a bounded cap (s < 1).  It is NOT a ray-geometry
// question, so the ray BVH cannot cull it.  Here the spheres get a tree of
// their own, built in the frame whose z axis is n (rows of R: u1, u2, n) over
// boxes c' +- r_e, and a shadow ray becomes a cone query from R o (device:
// bvh_trace<true>): a child is entered iff its top is not below the origin
// (tz >= 0), its lateral distance d from the origin satisfies
// d^2 <= max(0, k) tz^2, and for s < 1 its bottom is within
// r_e / sqrt(1 - s^2).  Every candidate is then tested with the exact
// reference arithmetic; the tree only decides which spheres are tested.
// Conservative margins: the computed discriminant's error, up to ~2^-21
// (1 + s^2) D^2, grows r^2 by 2^-18 (1 + s^2) D^2 (r_e), boxes grow by 2^-16 D,
// k is rounded up.  Returns false if the direction or the geometry is not
// finite, or the scene is so large that one ulp of B reaches epsilon (then
// the h < 0 side is no longer safe): the caller falls back to the scan.
bool dir_tree(const AccelInput &in, const AccelOpts &o, int threads, const LightK &lt, double D,
              std::vector<rtbvh::NodeDev> &nodes, std::vector<float4> &rec, DirK &out, int &max_stack) {
    for (int k = 0; k < 9; k++) out.R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
    out.root = -1;
    out.cone_k = 0.0f;
    out.cone_h = INFINITY;
    const double dx = lt.sdir[0], dy = lt.sdir[1], dz = lt.sdir[2];
    const double sl = std::sqrt(dx * dx + dy * dy + dz * dz);
    if (!std::isfinite(sl) || !(sl > 0.0)) return false;
    if (std::ldexp(2.0 * sl * D, -23) >= 0.5 * (double)in.eps) return false;
    const double n[3] = {dx / sl, dy / sl, dz / sl};
    // u1 perpendicular to n (cross with the axis least aligned with n), u2 = n x u1
    int ax = 0;
    for (int k = 1; k < 3; k++)
        if (std::fabs(n[k]) < std::fabs(n[ax])) ax = k;
    double e[3] = {0, 0, 0};
    e[ax] = 1.0;
    double u1[3] = {n[1] * e[2] - n[2] * e[1], n[2] * e[0] - n[0] * e[2], n[0] * e[1] - n[1] * e[0]};
    const double l1 = std::sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
    for (double &v : u1) v /= l1;
    const double u2[3] = {n[1] * u1[2] - n[2] * u1[1], n[2] * u1[0] - n[0] * u1[2], n[0] * u1[1] - n[1] * u1[0]};
    for (int k = 0; k < 3; k++) {
        out.R[k] = (float)u1[k];
        out.R[3 + k] = (float)u2[k];
        out.R[6 + k] = (float)n[k];
    }
    // the device rotates with the float R: boxes are computed with it too
    // (its rounding of R o, ~2^-22 D, is far inside the 2^-16 D margins)
    double R[9];
    for (int k = 0; k < 9; k++) R[k] = out.R[k];
    const double pad = std::ldexp(D, -16);
    const double s2 = sl * sl;
    std::vector<rtbvh::Prim> P;
    double re_max = 0.0;
    for (const auto &src : in.prims) {
        if (!src.sphere) continue;
        const double c[3] = {src.c[0], src.c[1], src.c[2]};
        const double r = std::fabs((double)src.r);
        if (!std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]) || !std::isfinite(r)) return false;
        const double re = std::sqrt(r * r + std::ldexp((1.0 + s2) * D * D, -18)) + 2.0 * pad;
        re_max = std::max(re_max, re);
        rtbvh::Prim q;
        q.key = src.key;
        q.cost = 1.0f;
        for (int k = 0; k < 3; k++) {
            const double cr = R[3 * k] * c[0] + R[3 * k + 1] * c[1] + R[3 * k + 2] * c[2];
            q.box.lo[k] = std::nextafter((float)(cr - re), -INFINITY);
            q.box.hi[k] = std::nextafter((float)(cr + re), INFINITY);
            q.c[k] = (float)cr;
        }
        P.push_back(q);
    }
    if (P.empty()) return true;                          // root -1: no sphere can shadow
    out.cone_k = std::nextafter((float)(std::max(0.0, s2 - 1.0) * (1.0 + std::ldexp(1.0, -16))), INFINITY);
    if (s2 < 1.0) out.cone_h = std::nextafter((float)(re_max / std::sqrt(1.0 - s2) + pad), INFINITY);
    rtbvh::Result Rb;
    rtbvh::Result4 Q;
    if (!build_wide(o, threads, P, Rb, Q, nullptr) || Q.max_stack > kStackMax) return false;
    max_stack = Q.max_stack;
    const int nf = in.nf;
    bool ok = rtbvh::leaf_records(
        Q, Rb.keys, [](int32_t) { return false; },
        [&](int32_t k) {
            float kb;
            memcpy(&kb, &k, sizeof kb);
            rec.push_back(in.sscan[k - nf]);
            rec.push_back(make_float4(kb, in.ofac[k], 0.0f, 0.0f));
            return 2;
        },
        rec.size());
    std::vector<rtbvh::NodeDev> QQ;
    if (!ok || !rtbvh::quantize(Q, QQ, threads)) return false;
    const int base = (int)nodes.size();
    for (auto &z : QQ) {
        for (auto &l : z.link) {
            if (l == rtbvh::kEmpty) l = rtbvh::kEmptyLeaf;
            else if (l >= 0) l += base;
        }
        nodes.push_back(z);
    }
    out.root = base;
    return true;
}

}  // namespace

int accel_threads() {
    int n = 1;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (const char *e = std::getenv("OMP_NUM_THREADS")) {
        const int k = std::atoi(e);
        if (k > 0) n = std::min(n, k);
    }
    return std::max(1, std::min(n, 16));
}

void accel_input(const rt_scene_desc *desc, AccelInput &in) {
    in = AccelInput();
    const int nf = desc->n_faces, ns = desc->n_spheres, nobj = nf + ns;
    in.nf = nf;
    in.ns = ns;
    in.eps = desc->epsilon;
    // --- faces: exact per-face invariants (TraceRay recomputes these per call)
    in.fscan.assign((size_t)nf * 5, make_float4(0, 0, 0, 0));
    in.fsh.assign((size_t)nf, FaceShadeK{});
    in.objs.assign((size_t)nobj, ObjK{});
    in.ofac.assign((size_t)nobj, 0.0f);
    auto fill_obj = [&](int k, const rt_material &m, int tex, int is_sphere) {
        ObjK &o = in.objs[k];
        for (int c = 0; c < 3; c++) o.dif[c] = m.diffuse[c], o.spc[c] = m.specular[c];
        o.ka = m.ka, o.kd = m.kd, o.ks = m.ks, o.n = m.n, o.opacity = m.opacity, o.eta = m.eta;
        o.tex = tex;
        o.is_sphere = is_sphere;
        in.ofac[k] = (float)(1.0 - (double)m.opacity);
        if (m.ks > 0.0f || (m.opacity < 1.0f && m.eta > 0.0f)) in.secondary = true;
    };
    for (int i = 0; i < nf; i++) {
        const rt_face_desc &F = desc->faces[i];
        V3 v0 = f3(F.v[0]), v1 = f3(F.v[1]), v2 = f3(F.v[2]);
        V3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
        V3 n = vnorm(vcross(e1, e2));                         // main.cpp:537-539
        float D = -vdot(n, v0);
        float d11 = vdot(e1, e1), d12 = vdot(e1, e2), d22 = vdot(e2, e2);
        float det = (d11 * d22 - d12 * d12);
        in.fscan[5 * i + 0] = make_float4(v0.x, v0.y, v0.z, D);
        in.fscan[5 * i + 1] = make_float4(n.x, n.y, n.z, det);
        in.fscan[5 * i + 2] = make_float4(e1.x, e1.y, e1.z, d11);
        in.fscan[5 * i + 3] = make_float4(e2.x, e2.y, e2.z, d22);
        in.fscan[5 * i + 4] = make_float4(d12, 0.0f, 0.0f, 0.0f);
        FaceShadeK &fs = in.fsh[i];
        for (int k = 0; k < 3; k++) {
            V3 vn = vnorm(f3(F.vn[k]));
            fs.vn[k][0] = vn.x, fs.vn[k][1] = vn.y, fs.vn[k][2] = vn.z;
            for (int c = 0; c < 2; c++) {
                float t = F.vt[k][c];
                fs.vt[k][c] = (t < 0.0f) ? 0.0f : ((1.0f < t) ? 1.0f : t);
            }
        }
        fs.smooth = F.smooth;
        fill_obj(i, F.mat, F.texture, 0);
    }
    // BVH sources (padding is applied per build, it depends on the eye)
    in.prims.reserve((size_t)nobj);
    for (int i = 0; i < nf; i++) {
        PrimSrc ps{};
        ps.key = i;
        ps.sphere = false;
        const rt_face_desc &F = desc->faces[i];
        for (int k = 0; k < 3; k++) {
            ps.lo[k] = std::min(F.v[0][k], std::min(F.v[1][k], F.v[2][k]));
            ps.hi[k] = std::max(F.v[0][k], std::max(F.v[1][k], F.v[2][k]));
        }
        float4 a = in.fscan[5 * i + 1], b2 = in.fscan[5 * i + 2], c2 = in.fscan[5 * i + 3];
        double det = a.w, d11 = b2.w, d22 = c2.w;
        ps.cond = det > 0 ? d11 * d22 / det : 1e30;
        for (int j = 0; j < 3; j++)
            for (int k = 0; k < 3; k++) ps.v[j][k] = F.v[j][k];
        in.prims.push_back(ps);
    }
    in.sscan.assign((size_t)ns, make_float4(0, 0, 0, 0));
    for (int i = 0; i < ns; i++) {
        const rt_sphere_desc &S = desc->spheres[i];
        in.sscan[i] = make_float4(S.center[0], S.center[1], S.center[2], S.radius);
        fill_obj(nf + i, S.mat, S.texture, 1);
        PrimSrc ps{};
        ps.key = nf + i;
        ps.sphere = true;
        for (int k = 0; k < 3; k++) {
            ps.c[k] = S.center[k];
            ps.lo[k] = S.center[k] - std::fabs(S.radius);
            ps.hi[k] = S.center[k] + std::fabs(S.radius);
        }
        ps.r = S.radius;
        in.prims.push_back(ps);
    }
    for (int k = 0; k < 3; k++) in.scene_lo[k] = INFINITY, in.scene_hi[k] = -INFINITY;
    for (const auto &ps : in.prims)
        for (int k = 0; k < 3; k++) {
            if (std::isfinite(ps.lo[k])) in.scene_lo[k] = std::min(in.scene_lo[k], ps.lo[k]);
            if (std::isfinite(ps.hi[k])) in.scene_hi[k] = std::max(in.scene_hi[k], ps.hi[k]);
        }
    for (int k = 0; k < 3; k++)
        if (!(in.scene_lo[k] <= in.scene_hi[k])) in.scene_lo[k] = in.scene_hi[k] = 0.0f;
    for (float f : in.ofac) in.nan_fac |= std::isnan(f);
    in.lights.assign((size_t)desc->n_lights, LightK{});
    for (int i = 0; i < desc->n_lights; i++) {
        const rt_light_desc &L = desc->lights[i];
        LightK &k = in.lights[i];
        memset(&k, 0, sizeof k);
        for (int c = 0; c < 3; c++) k.xyz[c] = L.xyz[c], k.col[c] = L.color[c];
        k.w = L.w;
        V3 dir = f3(L.xyz);
        V3 Ld = vmul(vnorm(dir), -1.0f);
        V3 sd = vmul(dir, -1.0f);
        k.L[0] = Ld.x, k.L[1] = Ld.y, k.L[2] = Ld.z;
        k.sdir[0] = sd.x, k.sdir[1] = sd.y, k.sdir[2] = sd.z;
    }
    // Density: the objects a straight line across the scene's box meets on
    // average -- total cross-section (spheres pi r^2, triangles area / 2,
    // averaged over directions) per volume, times the box diagonal (C3: ~3,
    // C5: ~200); it decides the origin-leaf pass (rt_scene.cpp).
    double xs = 0.0, vol = 1.0, diag2 = 0.0;
    for (int i = 0; i < nf; i++) {
        V3 c = vcross(f3(&in.fscan[5 * i + 2].x), f3(&in.fscan[5 * i + 3].x));
        xs += 0.25 * std::sqrt((double)c.x * c.x + (double)c.y * c.y + (double)c.z * c.z);
    }
    for (int i = 0; i < ns; i++) xs += kPi * (double)in.sscan[i].w * (double)in.sscan[i].w;
    for (int k = 0; k < 3; k++) {
        const double e = (double)in.scene_hi[k] - (double)in.scene_lo[k];
        vol *= e;
        diag2 += e * e;
    }
    in.crossings = vol > 0.0 && std::isfinite(xs) ? xs / vol * std::sqrt(diag2) : 0.0;
}

double distance_bound(const AccelInput &in, const float eye[3]) {
    double diag2 = 0, far2 = 0, mag = 0;
    for (int k = 0; k < 3; k++) {
        double e = in.scene_hi[k] - in.scene_lo[k];
        diag2 += e * e;
        double a = std::fabs(eye[k] - in.scene_lo[k]), b = std::fabs(eye[k] - in.scene_hi[k]);
        far2 += std::max(a, b) * std::max(a, b);
        mag = std::max(mag, std::max(std::fabs((double)in.scene_lo[k]), std::fabs((double)in.scene_hi[k])));
        mag = std::max(mag, std::fabs((double)eye[k]));
    }
    return std::max(std::sqrt(diag2), std::sqrt(far2)) + mag + 1.0;
}

void build_accel(const AccelInput &in, double D, const AccelOpts &o, AccelTree &out) {
    out = AccelTree();
    const int threads = o.threads > 0 ? o.threads : accel_threads();
    out.threads = threads;
    auto t0 = Clock::now();
    std::vector<rtbvh::Prim> P(in.prims.size());
    rtbvh::parallel_ranges(P.size(), threads, [&](size_t i0, size_t i1) {
      for (size_t i = i0; i < i1; i++) {
        const auto &src = in.prims[i];
        rtbvh::Prim &q = P[i];
        q.key = src.key;
        if (!src.sphere) {
            double pad = std::ldexp(D, -16) * std::max(1.0, src.cond);
            for (int k = 0; k < 3; k++) {
                q.box.lo[k] = (float)(src.lo[k] - pad);
                q.box.hi[k] = (float)(src.hi[k] + pad);
                q.c[k] = 0.5f * (src.lo[k] + src.hi[k]);
            }
            q.cost = 3.0f;
        } else {
            double r = std::fabs((double)src.r);
            double rr = std::sqrt(r * r + std::ldexp(D * D, -18)) + std::ldexp(D, -16);
            for (int k = 0; k < 3; k++) {
                q.box.lo[k] = (float)(src.c[k] - rr);
                q.box.hi[k] = (float)(src.c[k] + rr);
                q.c[k] = src.c[k];
            }
            q.cost = 1.0f;
        }
        // float rounding of the padded box must not shrink it
        for (int k = 0; k < 3; k++) {
            q.box.lo[k] = std::nextafter(q.box.lo[k], -INFINITY);
            q.box.hi[k] = std::nextafter(q.box.hi[k], INFINITY);
            if (!std::isfinite(q.box.lo[k]) || !std::isfinite(q.box.hi[k])) {
                q.box.lo[k] = -INFINITY;   // NaN/inf geometry: a box every ray enters
                q.box.hi[k] = INFINITY;
            }
        }
      }
    });
    // (off by default: 2 references per face took the benchmark's C4 from
    // 14.11 to 13.36 ms, but four other seeds of its generator -2.8 ... +5.1 %,
    // and C3 -1.0 %; a split-gain of 0.8 or 0.95 instead of 0.9 lost on C4
    // itself -- the tree's response is not a property of the scene kind,
    // profiles/r05/ab/presplit_*)
    const int presplit = std::max(0, o.presplit);
    out.presplit = presplit;
    if (presplit > 1) {
        // faces with a shadow factor of exactly 0 or 1 and finite boxes: their
        // pieces (split_face), in primitive order (the same tree for every
        // thread count)
        std::vector<rtbvh::Prim> S;
        S.reserve(P.size());
        std::vector<ClipBox> pieces;
        for (size_t i = 0; i < P.size(); i++) {
            const auto &src = in.prims[i];
            const float fac = src.sphere ? 0.5f : in.ofac[(size_t)src.key];
            bool finite = true;
            for (int k = 0; k < 3; k++) finite &= std::isfinite(P[i].box.lo[k]) && std::isfinite(P[i].box.hi[k]);
            if (src.sphere || !finite || !(fac == 0.0f || fac == 1.0f)) {
                S.push_back(P[i]);
                continue;
            }
            split_face(src.v, presplit, pieces);
            const double pad = std::ldexp(D, -16) * std::max(1.0, src.cond);
            for (const ClipBox &c : pieces) {
                rtbvh::Prim q = P[i];
                for (int k = 0; k < 3; k++) {
                    q.box.lo[k] = std::nextafter((float)(c.lo[k] - pad), -INFINITY);
                    q.box.hi[k] = std::nextafter((float)(c.hi[k] + pad), INFINITY);
                    q.c[k] = (float)(0.5 * (c.lo[k] + c.hi[k]));
                }
                S.push_back(q);
            }
        }
        P.swap(S);
    }
    out.refs = (long long)P.size();
    out.ms[0] = ms_since(t0);
    rtbvh::Result R;
    rtbvh::Result4 Q;
    bool ok = P.empty() || build_wide(o, threads, P, R, Q, out.ms, &out.sah);
    // leaf records: face = its 5 scan words with (key, shadow factor) in the
    // last one's y, z; sphere = (centre, r), (key, shadow factor, 0, 0)
    t0 = Clock::now();
    std::vector<float4> &rec = out.rec;
    rec.reserve((size_t)in.nf * 5 + (size_t)in.ns * 2 + 3);
    const int nf = in.nf;
    if (ok && !Q.nodes.empty())
        ok = rtbvh::leaf_records(Q, R.keys, [nf](int32_t k) { return k < nf; }, [&](int32_t k) {
            float kb;
            memcpy(&kb, &k, sizeof kb);
            float fac = in.ofac[k];
            if (k < nf) {
                for (int j = 0; j < 5; j++) rec.push_back(in.fscan[5 * (size_t)k + j]);
                rec.back().y = kb;
                rec.back().z = fac;
                return 5;
            }
            rec.push_back(in.sscan[k - nf]);
            rec.push_back(make_float4(kb, fac, 0.0f, 0.0f));
            return 2;
        });
    rec.resize(rec.size() + 3, make_float4(0.0f, 0.0f, 0.0f, 0.0f));   // 5-word reads of a last sphere
    // every object's leaf in the main tree (the origin-leaf pass, bvh_trace)
    out.objleaf.assign((size_t)std::max(1, nf + in.ns), rtbvh::kEmptyLeaf);
    if (ok)
        for (const auto &n : Q.nodes)
            for (int32_t l : n.link) {
                if (l >= 0 || l == rtbvh::kEmpty) continue;
                const int v = -l - 1, nfc = (v >> 4) & 15, count = v & 15;
                size_t off = (size_t)(v >> 8);
                for (int k = 0; k < count; k++) {
                    int32_t key;
                    if (k < nfc) {
                        memcpy(&key, &rec[off + 4].y, sizeof key);
                        off += 5;
                    } else {
                        memcpy(&key, &rec[off + 1].x, sizeof key);
                        off += 2;
                    }
                    out.objleaf[(size_t)key] = l;
                }
            }
    out.ms[3] = ms_since(t0);
    t0 = Clock::now();
    std::vector<rtbvh::NodeDev> &QQ = out.nodes;
    if (ok && !Q.nodes.empty() && !rtbvh::quantize(Q, QQ, threads)) ok = false;   // non-finite geometry: scan
    for (auto &z : QQ)                                  // device form: unused slot -> the empty leaf
        for (auto &l : z.link)
            if (l == rtbvh::kEmpty) l = rtbvh::kEmptyLeaf;
    out.ms[4] = ms_since(t0);
    // the spill area is sized for the deepest tree (kStackMax: far beyond any
    // tree the builder's depth cap allows)
    ok = ok && !Q.nodes.empty() && Q.max_stack <= kStackMax;
    // directional lights in a scene with spheres: shadow-region trees, after
    // the main tree in the same node and record arrays
    t0 = Clock::now();
    out.dirk.assign(in.lights.size(), DirK{});
    int dir_mode = 0;
    int stack_all = Q.max_stack;                 // deepest stack over the main and the cone trees
    if (ok && in.ns > 0) {
        rec.resize(rec.size() - 3);                  // the 3 padding words go after the last tree
        for (size_t l = 0; l < in.lights.size(); l++) {
            if (in.lights[l].w != 0.0f) continue;
            if (dir_mode == 0) dir_mode = 2;
            int st = 0;
            if (!dir_tree(in, o, threads, in.lights[l], D, QQ, rec, out.dirk[l], st)) dir_mode = 1;
            stack_all = std::max(stack_all, st);
        }
        rec.resize(rec.size() + 3, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    }
    out.ms[5] = ms_since(t0);
    // device links: an inner node's link is its byte offset in the node array
    // (the kernel fetches a node with buffer loads at that offset: no address
    // arithmetic per visit), leaf links stay as they are
    if (ok && QQ.size() * sizeof(rtbvh::NodeDev) > (size_t)INT32_MAX) ok = false;
    if (ok) {
        for (auto &z : QQ)
            for (auto &l : z.link)
                if (l >= 0) l *= (int32_t)sizeof(rtbvh::NodeDev);
        for (auto &d : out.dirk)
            if (d.root >= 0) d.root *= (int)sizeof(rtbvh::NodeDev);
    }
    out.ok = ok;
    out.dir_mode = dir_mode;
    out.depth = Q.depth;
    out.max_stack = Q.max_stack;
    out.stack_all = stack_all;
    out.main_nodes = (long long)Q.nodes.size();
}

}  // namespace rt
