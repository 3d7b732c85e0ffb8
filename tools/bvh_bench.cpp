// Host BVH build of a scene file, timed per phase and checked for
// determinism: the build on T threads must give the serial build's trees
// bit for bit (rt_bvh.h Builder / quantize).  No GPU is used.
//
//   make -C simple-raytracer_amd bvh_bench
//   simple-raytracer_amd/lib/bvh_bench scene.txt [threads] [reps] [presplit]
//
// Prints one JSON line: primitives, nodes, per-phase ms (best of reps) for
// the serial and the threaded build, "identical" and the tree's hash.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_accel.h"
#include "rt_host.h"

using namespace rt;

static bool same(const AccelTree &a, const AccelTree &b) {
    auto eq = [](const void *x, const void *y, size_t n) { return n == 0 || std::memcmp(x, y, n) == 0; };
    return a.ok == b.ok && a.nodes.size() == b.nodes.size() && a.rec.size() == b.rec.size() &&
           a.objleaf.size() == b.objleaf.size() && a.dirk.size() == b.dirk.size() && a.dir_mode == b.dir_mode &&
           a.depth == b.depth && a.max_stack == b.max_stack && a.stack_all == b.stack_all &&
           eq(a.nodes.data(), b.nodes.data(), a.nodes.size() * sizeof(a.nodes[0])) &&
           eq(a.rec.data(), b.rec.data(), a.rec.size() * sizeof(a.rec[0])) &&
           eq(a.objleaf.data(), b.objleaf.data(), a.objleaf.size() * sizeof(a.objleaf[0])) &&
           eq(a.dirk.data(), b.dirk.data(), a.dirk.size() * sizeof(a.dirk[0]));
}

// FNV-1a over the uploaded arrays: the tree's identity across builds
static unsigned long long tree_hash(const AccelTree &t) {
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
        const unsigned char *b = static_cast<const unsigned char *>(p);
        for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    };
    mix(t.nodes.data(), t.nodes.size() * sizeof(t.nodes[0]));
    mix(t.rec.data(), t.rec.size() * sizeof(t.rec[0]));
    mix(t.objleaf.data(), t.objleaf.size() * sizeof(t.objleaf[0]));
    mix(t.dirk.data(), t.dirk.size() * sizeof(t.dirk[0]));
    return h;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s scene.txt [threads] [reps]\n", argv[0]);
        return 2;
    }
    const int threads = argc > 2 ? std::atoi(argv[2]) : accel_threads();
    const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
    rth_scene *hs = nullptr;
    char msg[512] = {0};
    using Clock = std::chrono::steady_clock;
    auto t0 = Clock::now();
    if (rth_parse_file(argv[1], &hs, msg, sizeof msg) != 0) {
        std::fprintf(stderr, "parse failed: %s\n", msg);
        return 1;
    }
    const double parse_ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    const rt_scene_desc *desc = rth_desc(hs);
    rt_camera cam;
    rth_camera(hs, rth_width(hs), rth_height(hs), &cam);
    t0 = Clock::now();
    AccelInput in;
    accel_input(desc, in);
    const double input_ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    const double D = distance_bound(in, cam.eye);
    const int presplit = argc > 4 ? std::atoi(argv[4]) : 0;
    AccelTree ref, par;
    double best[2] = {1e30, 1e30}, ph[2][6];
    for (int r = 0; r < reps; r++) {
        for (int v = 0; v < 2; v++) {
            AccelOpts o;
            o.threads = v == 0 ? 1 : threads;
            o.presplit = presplit;
            AccelTree &T = v == 0 ? ref : par;
            auto t = Clock::now();
            build_accel(in, D, o, T);
            const double ms = std::chrono::duration<double, std::milli>(Clock::now() - t).count();
            if (ms < best[v]) {
                best[v] = ms;
                for (int k = 0; k < 6; k++) ph[v][k] = T.ms[k];
            }
        }
    }
    const bool ident = same(ref, par);
    auto phases = [&](int v) {
        static char b[2][256];
        std::snprintf(b[v], sizeof b[v],
                      "{\"prims\": %.3f, \"binary\": %.3f, \"collapse\": %.3f, \"records\": %.3f, \"quantize\": %.3f, "
                      "\"cone_trees\": %.3f}",
                      ph[v][0], ph[v][1], ph[v][2], ph[v][3], ph[v][4], ph[v][5]);
        return (const char *)b[v];
    };
    std::printf("{\"scene\": \"%s\", \"faces\": %d, \"spheres\": %d, \"lights\": %d, \"parse_ms\": %.3f, "
                "\"input_ms\": %.3f, \"nodes\": %zu, \"main_nodes\": %lld, \"ok\": %d, \"threads\": %d, "
                "\"serial_ms\": %.3f, \"threaded_ms\": %.3f, \"serial_phases_ms\": %s, \"threaded_phases_ms\": %s, "
                "\"identical\": %s, \"hash\": \"%016llx\", \"node_bytes\": %zu, "
                "\"presplit\": %d, \"refs\": %lld, \"sah\": %.4f}\n",
                argv[1], in.nf, in.ns, (int)in.lights.size(), parse_ms, input_ms, ref.nodes.size(), ref.main_nodes,
                ref.ok ? 1 : 0, par.threads, best[0], best[1], phases(0), phases(1), ident ? "true" : "false", tree_hash(ref),
                sizeof(rtbvh::NodeDev), ref.presplit, ref.refs, ref.sah);
    rth_free(hs);
    return ident ? 0 : 3;
}
