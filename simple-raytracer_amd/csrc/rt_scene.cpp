// rt_scene.cpp -- host side of librt_hip.so: scene upload (the device layout
// of rt_device.h), BVH build and upload (rt_bvh.h), render slots, and the C ABI
// of include/rt_hip.h.  The kernels are in rt_kernels.hip.
//
// The seam this replaces: create_view_window_and_ray_trace (main.cpp:607,
// :670-767) and its implicit inputs from the global `environment`
// (main.cpp:58, src/definitions.h:304-311).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "rt_accel.h"
#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_hip.h"

using namespace rt;

// One render in flight: its work counter, counters, ShadeRay frame buffer and
// events.  A scene has `inflight` of them (rt_scene_set_option "inflight"):
// with one, a render runs on the caller's stream; with more, render k runs on
// slot k mod n's own stream, ordered against the caller's stream by events, so
// that renders issued on different caller streams (independent frames) overlap:
// the next frame's workgroups fill the CUs that the current frame's tail leaves
// idle.
struct RenderSlot {
    hipStream_t stream = nullptr;      // slots > 1 only (high priority: its own HW queue pool)
    hipEvent_t ev_in = nullptr;        // caller stream -> slot stream
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    unsigned long long *stats = nullptr;
    void *d_frames = nullptr;          // ShadeRay frames of the launch
    size_t frames_cap = 0;
    bool used = false;                 // ev1 marks a render issued through this slot
};

struct rt_scene {
    int device = 0;
    hipStream_t stream = nullptr;
    Params base{};
    std::vector<void *> allocs;
    float *dev_out = nullptr;          // staging buffer when the caller passes host memory
    size_t dev_out_bytes = 0;
    int *dev_pix = nullptr;            // rt_render_pixels: the pixel list on the device
    size_t dev_pix_bytes = 0;
    std::vector<RenderSlot> slots;     // slots[0] always exists
    int next_slot = 0;                 // slot of the next render
    int last_slot = 0;                 // slot of the last render
    int num_cu = 0;
    size_t max_lds = 64 * 1024;        // the device's LDS limit per workgroup
    size_t lds_bytes = 0;
    long long opt_lds = -1;            // -1 auto, 0 off, 1 on
    long long opt_lds_stack = -1;      // BVH stack entries in LDS (-1: by depth, launch)
    double crossings = 0.0;            // objects a line across the scene meets on average (org_first)
    int org_first_auto = 0;            // org_first by that density
    long long opt_grid = 0;            // blocks (0 = occupancy-derived)
    long long opt_chunk = -1;          // refill chunk (-1: default, chunk_for)
    long long opt_refill_min = -1;     // idle lanes before a refill (-1: by the scene, refill_for)
    long long opt_work_parts = -1;     // work item bands with a counter each (-1: one per XCD when the launch allows)
    bool secondary = false;            // some material reflects (ks > 0) or refracts (opacity < 1, eta > 0)
    long long opt_reserve = 0;         // occupancy-derived grid: block slots left free for other kernels
    long long opt_accel = -1;          // -1 auto, 0 brute-force scan, 1 BVH
    long long opt_bvh_leaf = 8;        // SAH max leaf size
    long long opt_bvh_presplit = 0;    // references per opaque face at most (rt_accel.cpp presplit)
    long long opt_bvh_collapse = 1;    // binary -> 4-wide: 0 greedy (largest area first), 1 SAH-optimal DP
    long long opt_bvh_node = 500;      // DP collapse: cost of a 4-wide node visit, x1000 of a sphere test
                                       // (A/B, C3: 0.25 / 0.5 / 0.75 / 1 / 2 -> +0.6 / +0.5 / +0.5 / +0.2 / -1.7 %)
    long long opt_fail_bvh_upload = 0; // test hook: the next BVH uploads fail (RT_E_NOMEM)
    AccelInput in;                     // host arrays + BVH sources (rt_accel.h)
    long long opt_bvh_threads = 0;     // host threads of the BVH build (0: automatic, 1: serial)
    long long opt_counters = kCounters;  // 1: the counting kernel (rt_stats' rays, events, tests); 0: none
    long long opt_frame_share = -1;    // the occupancy-sized grid / this: frames in flight that run side by
                                       // side (-1 auto: kFrameShare for small frames with inflight > 1, else 1)
    long long opt_recursive = 0;       // test hook: 1 forces the recursive instantiation (MAXF by depth) on a
                                       // scene without reflecting / refracting materials (no last-light skip)
    int last_light_skip_auto = 0;      // Params::last_light_skip when exact for the scene
    double bvh_D = -1.0;               // distance bound the current BVH was padded for
    float4 *d_bvh = nullptr;
    float4 *d_leafrec = nullptr;
    DirK *d_dirk = nullptr;            // per light: shadow-region tree (directional lights)
    int *d_objleaf = nullptr;          // per object: its leaf's link in the main tree
    AccelTree last_tree_ms;            // phase times of the last build (bvh_phase_ms)

    int bvh_depth = 0;
    int bvh_stack = 0;
    int ovf_stride = kSpill;           // spilled BVH stack entries per lane (Params::ovf_stride)
    bool bvh_ok = false;
    double bvh_build_ms = 0.0;         // host time of the last BVH (re)build
    long long last_blocks_per_cu = 0, last_grid = 0, last_lds = 0, last_mode = -1;
    long long last_org_first = 0, last_stack_cap = 0, last_lights_in_lds = 0, last_work_parts = 0, last_maxf = 0;
    long long bvh_nodes = 0;
    bool last_valid = false;
};

namespace {

const char *kErr[] = {"ok", "invalid argument", "no such HIP device", "HIP runtime error", "out of device memory",
                      "unsupported"};

// Streams made ahead of the scenes by rt_device_init (the first stream of a
// process costs ~10 ms: its hardware queue), taken by rt_scene_create and
// given back by rt_scene_destroy.
std::mutex g_pool_mu;
std::vector<std::pair<int, hipStream_t>> g_stream_pool;

hipStream_t take_stream(int device) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_stream_pool.size(); i++)
        if (g_stream_pool[i].first == device) {
            hipStream_t st = g_stream_pool[i].second;
            g_stream_pool.erase(g_stream_pool.begin() + (long)i);
            return st;
        }
    return nullptr;
}
bool pool_has(int device) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (const auto &e : g_stream_pool)
        if (e.first == device) return true;
    return false;
}
void give_stream(int device, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_stream_pool.emplace_back(device, st);
}

// RT_TIMING=1 in the environment: the steps of scene creation and of the
// first renders on the host clock, to stderr (the one-shot CLI's fixed costs,
// DESIGN.md §7a)
struct StepTimer {
    bool on = std::getenv("RT_TIMING") != nullptr;
    const char *what;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    explicit StepTimer(const char *w) : what(w) {}
    void mark(const char *step) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[rt timing] %s %s %.3f ms\n", what, step,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// Host staging of several device arrays packed into one allocation, each at
// a 256-B aligned offset (at least one element's room, as the arrays were
// allocated one by one before round 5)
struct Arena {
    std::vector<char> host;
    size_t reserve(size_t bytes) {
        const size_t off = (host.size() + 255) / 256 * 256;
        host.resize(off + std::max<size_t>(16, bytes), 0);
        return off;
    }
    template <typename T>
    size_t add(const std::vector<T> &v) {
        const size_t off = reserve(std::max<size_t>(1, v.size()) * sizeof(T));
        if (!v.empty()) std::memcpy(host.data() + off, v.data(), v.size() * sizeof(T));
        return off;
    }
};


// Dynamic LDS of render_kernel: the per-lane shading state, the mode's region
// (BVH stacks or the staged primitives), then the lights when they all fit
// under the device's per-workgroup LDS limit (else the kernel reads them from
// device memory, Params::lights_in_lds: a scene with thousands of lights
// still renders).
size_t mode_region_end(const rt_scene *s, int mode, const Params &p) {
    size_t shade = (size_t)kLdsHotWords * kBlock * sizeof(float);    // per-lane shading state
    if (mode == MODE_SCAN_LDS) return shade + s->lds_bytes;
    if (mode == MODE_BVH) return shade + (size_t)p.stack_cap * kBlock * sizeof(int);
    return shade;
}
// The launch's dynamic LDS; decides Params::lights_in_lds: the lights are
// staged when they fit under the limit and do not cost a resident workgroup
// per CU (by the occupancy calculator), else they come from device memory.
size_t mode_lds_bytes(const rt_scene *s, int maxf, int mode, Params &p) {
    const size_t end = mode_region_end(s, mode, p);
    const size_t with = end + (size_t)p.nl * sizeof(LightK);
    p.lights_lds = (int)(end / sizeof(float4));
    const bool cnt = s->opt_counters != 0;
    p.lights_in_lds =
        with <= s->max_lds && render_blocks_per_cu(maxf, mode, cnt, with) >= render_blocks_per_cu(maxf, mode, cnt, end);
    return p.lights_in_lds ? with : end;
}

// Work items a wave takes from the pixel counter at a time: by default
// exactly its idle lanes' count.  A whole 8x8 tile per wave (64) was +5 % on
// C3 while every idle lane was refilled at once; with the deferred refill
// (refill_for) it is -3 % on C3 and -10 % on C4, and it never changes the
// image (profiles/r02/ab_chunk_auto.txt, ab_refill_min.txt).
static unsigned chunk_for(const rt_scene *s) {
    return s->opt_chunk >= 0 ? (unsigned)s->opt_chunk : 0u;
}

// How many lanes of a wave must be idle before it refills them.  With only
// primary and shadow rays, a pixel lasts a few trace steps: the whole wave
// starts 64 pixels together and finishes them before the next batch (C4
// 10.9 G rays/s against 10.7 at 48 and 8.3 at 1).  With reflection /
// refraction, 32 up to depth 4 (C3 +0.8 % over 40 in 4 rounds, C3G +0.9 %,
// C3D -0.2 %) and 48 for deeper shade trees, whose pixels live longer (C5
// +0.8 % over 40, -1.6 % at 32; profiles/r02/ab_refill_min.txt, ab_gate.txt).
static unsigned refill_for(const rt_scene *s, const Params &p) {
    if (s->opt_refill_min > 0) return (unsigned)s->opt_refill_min;
    if (!s->secondary || p.depth <= 0) return 64u;
    return p.depth > 4 ? 48u : 32u;
}

hipError_t launch_one(rt_scene *s, RenderSlot &slot, const Params &p, int maxf, int mode, hipStream_t st, bool dry) {
    StepTimer tm(dry ? "prepare" : "launch");
    Params pl = p;
    size_t shm = mode_lds_bytes(s, maxf, mode, pl);
    int nb = render_blocks_per_cu(maxf, mode, s->opt_counters != 0, shm);
    tm.mark("occupancy");
    if (nb < 1) nb = 1;
    long long grid = s->opt_grid > 0 ? s->opt_grid : (long long)nb * s->num_cu - s->opt_reserve;
    // Short frames in flight (option inflight > 1, at most kFrameShareItems
    // work items per lane of the occupancy-sized grid: C3's rows of one rank
    // at N = 2 / 4 / 8, 25.6 / 12.8 / 6.4 per lane) run side by side on a
    // share of the CUs each: a frame's tail -- its waves finishing the pixels
    // they hold once the work is gone, a workgroup's slots freed only when its
    // four waves are done -- then idles only its own share while the other
    // frames go on.  C3 pipelined at half the grid: N = 8 1.763 -> 1.649 ms
    // per frame (a third: 1.663, a quarter: 1.752), N = 4 3.19 -> 3.05,
    // N = 2 6.09 -> 5.89; a whole C3 frame (51 per lane) gains nothing from
    // it (-1.1 % over 60 steps; profiles/r05/frame_share/)
    if (s->opt_grid <= 0) {
        const bool small = (unsigned long long)p.total <= (unsigned long long)grid * kBlock * kFrameShareItems;
        const long long share = s->opt_frame_share > 0 ? s->opt_frame_share
                                : s->slots.size() > 1 && small ? kFrameShare : 1;
        grid = std::max(1LL, grid / share);
    }
    long long need = ((long long)p.total + kBlock - 1) / kBlock;
    if (grid > need) grid = need;
    if (grid < 1) grid = 1;
    pl.chunk = chunk_for(s);
    pl.refill_min = refill_for(s, pl);
    // work bands: one per XCD (workgroup b runs on XCD b mod 8: its L2), unless
    // the launch is too small to give each band a workgroup (option work_parts)
    const unsigned parts = s->opt_work_parts > 0 ? (unsigned)s->opt_work_parts
                           : (grid >= kWorkPartsMax && p.total >= (unsigned)(kWorkPartsMax * kBlock))
                               ? (unsigned)kWorkPartsMax
                               : 1u;
    pl.work_shift = parts >= 8 ? 3 : parts >= 4 ? 2 : parts >= 2 ? 1 : 0;
    const size_t cold_bytes = (size_t)grid * kBlock * maxf * cold_frame_bytes(maxf);
    size_t fbytes = cold_bytes + (size_t)grid * kBlock * s->ovf_stride * sizeof(int);
    // recursive instantiations (dense_heads): the frame heads, [block][level]
    // [lane] 32 B per slot (head_split: 16-B heads, then as many 16-B stack
    // slots), after the spill area (Params::heads, LaneState::fr)
    const size_t heads_off = (fbytes + 255) / 256 * 256;
    if (dense_heads(maxf)) fbytes = heads_off + (size_t)grid * kBlock * maxf * kHeadInts * 4;
    if (slot.frames_cap < fbytes) {
        // (re)size every slot's buffer now, not each at its first use: a
        // frame pipeline then allocates once, in its first (warm-up) frame
        for (RenderSlot &r : s->slots) {
            if (r.frames_cap >= fbytes) continue;
            if (r.d_frames) (void)hipFree(r.d_frames);
            r.d_frames = nullptr;
            r.frames_cap = 0;
            if (hipMalloc(&r.d_frames, fbytes) != hipSuccess) return hipErrorOutOfMemory;
            r.frames_cap = fbytes;
        }
    }
    tm.mark("frames");
    pl.frames = slot.d_frames;
    pl.ovf = reinterpret_cast<int *>(static_cast<char *>(slot.d_frames) + cold_bytes);
    pl.heads = dense_heads(maxf) ? static_cast<char *>(slot.d_frames) + heads_off : nullptr;
    s->last_blocks_per_cu = nb;
    s->last_grid = grid;
    s->last_lds = (long long)shm;
    s->last_mode = mode;
    s->last_org_first = pl.org_first;
    s->last_stack_cap = pl.stack_cap;
    s->last_lights_in_lds = pl.lights_in_lds;
    s->last_work_parts = 1 << pl.work_shift;
    s->last_maxf = maxf;
    if (dry) return hipSuccess;                  // rt_scene_prepare: buffers only
    const hipError_t e = render_launch(maxf, mode, s->opt_counters != 0, pl, (unsigned)grid, shm, st);
    tm.mark("kernel launch (enqueue)");
    return e;
}

// (Re)build the BVH for distance bound D on the host (rt_accel.cpp) and
// upload it.
int build_bvh(rt_scene *s, double D) {
    const auto t0 = std::chrono::steady_clock::now();
    AccelOpts o;
    o.bvh_leaf = (int)s->opt_bvh_leaf;
    o.collapse = (int)s->opt_bvh_collapse;
    o.node_milli = (int)s->opt_bvh_node;
    o.threads = (int)s->opt_bvh_threads;
    o.presplit = (int)s->opt_bvh_presplit;
    AccelTree T;
    StepTimer tm("build_bvh");
    build_accel(s->in, D, o, T);
    tm.mark("host build");
    bool ok = T.ok;
    const std::vector<rtbvh::NodeDev> &QQ = T.nodes;
    const std::vector<float4> &rec = T.rec;
    const std::vector<DirK> &dirk = T.dirk;
    const std::vector<int32_t> &objleaf = T.objleaf;
    // The old tree stays valid until the new one is on the device: upload into
    // new buffers first, then swap (a failed rebuild leaves no dangling
    // pointers and no tree marked valid that is not there).
    float4 *nb = nullptr, *nr = nullptr;
    DirK *nd = nullptr;
    int *nl = nullptr;
    int rc = RT_OK;
    if (ok && s->opt_fail_bvh_upload) {        // test hook: as if the device allocation failed
        rc = RT_E_NOMEM;
        ok = false;
    }
    if (ok) {
        const size_t node_bytes = QQ.size() * sizeof(QQ[0]);
        const size_t dir_bytes = std::max<size_t>(1, dirk.size()) * sizeof(DirK);
        if (hipMalloc(&nb, node_bytes) != hipSuccess ||
            hipMalloc(&nr, std::max<size_t>(1, rec.size()) * sizeof(float4)) != hipSuccess ||
            hipMalloc(&nd, dir_bytes) != hipSuccess || hipMalloc(&nl, objleaf.size() * sizeof(int32_t)) != hipSuccess)
            rc = RT_E_NOMEM;
        else if (hipMemcpy(nb, QQ.data(), node_bytes, hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(nr, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess ||
                 (!dirk.empty() && hipMemcpy(nd, dirk.data(), dirk.size() * sizeof(DirK), hipMemcpyHostToDevice) !=
                                       hipSuccess) ||
                 hipMemcpy(nl, objleaf.data(), objleaf.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
            rc = RT_E_HIP;
        if (rc) {
            if (nb) (void)hipFree(nb);
            if (nr) (void)hipFree(nr);
            if (nd) (void)hipFree(nd);
            if (nl) (void)hipFree(nl);
            nb = nr = nullptr;
            nd = nullptr;
            nl = nullptr;
        }
    }
    // renders still queued may read the old tree: free it after they finish
    if (s->d_bvh || s->d_leafrec || s->d_dirk || s->d_objleaf) {
        (void)hipDeviceSynchronize();
        if (s->d_bvh) (void)hipFree(s->d_bvh);
        if (s->d_leafrec) (void)hipFree(s->d_leafrec);
        if (s->d_dirk) (void)hipFree(s->d_dirk);
        if (s->d_objleaf) (void)hipFree(s->d_objleaf);
    }
    s->d_bvh = nb;
    s->d_leafrec = nr;
    s->d_dirk = nd;
    s->d_objleaf = nl;
    s->base.objleaf = nl;
    s->base.bvh = nb;
    s->base.leafrec = nr;
    s->base.dirk = nd;
    s->base.dir_bf = T.dir_mode;
    tm.mark("upload");
    s->bvh_ok = ok && rc == RT_OK;
    s->bvh_D = rc == RT_OK ? D : -1.0;   // a failed upload is retried; an unusable tree (scan) is not
    s->bvh_depth = s->bvh_ok ? T.depth : 0;
    s->bvh_stack = s->bvh_ok ? T.max_stack : 0;
    // spill area per lane: every block of kSpill entries a stack can push out
    s->ovf_stride = s->bvh_ok ? (T.stack_all / kSpill + 1) * kSpill : kSpill;
    s->bvh_nodes = s->bvh_ok ? T.main_nodes : 0;
    s->last_tree_ms = AccelTree();
    for (int k = 0; k < 6; k++) s->last_tree_ms.ms[k] = T.ms[k];
    s->last_tree_ms.threads = T.threads;
    s->bvh_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int launch(rt_scene *s, RenderSlot &slot, Params &p, hipStream_t st, bool dry = false) {
    int depth = p.depth < 0 ? 0 : p.depth;
    int maxf = maxf_for(depth, s->secondary || (s->opt_recursive && depth > 0));
    if (maxf < 0) return RT_E_UNSUPPORTED;
    if (head_split(maxf) && p.nl > kSplitLightMax) maxf = 17;   // its meta's light index field (rt_device.h)
    int nobj = p.nf + p.ns;
    bool bvh = s->opt_accel == 1 || (s->opt_accel == -1 && nobj > 32);
    int mode = MODE_SCAN;
    if (bvh) {
        double D = distance_bound(s->in, p.eye);
        if (D > s->bvh_D) {
            int rc = build_bvh(s, std::max(D, 1.5 * s->bvh_D));
            if (rc) return rc;
        }
        if (s->bvh_ok) {
            mode = MODE_BVH;
            p.bvh = s->base.bvh;
            p.leafrec = s->base.leafrec;
            p.dirk = s->base.dirk;
            p.objleaf = s->base.objleaf;
            p.dir_bf = s->base.dir_bf;
            p.ovf_stride = s->ovf_stride;
        }
    }
    if (mode == MODE_SCAN) {
        bool lds = s->opt_lds == 1 || (s->opt_lds == -1 && s->lds_bytes <= 64 * 1024);
        if (s->lds_bytes > 64 * 1024) lds = false;
        if (lds) mode = MODE_SCAN_LDS;
    }
    if (mode == MODE_SCAN_LDS && mode_region_end(s, MODE_SCAN_LDS, p) > s->max_lds) mode = MODE_SCAN;
    // BVH stack entries in LDS (option lds_stack, else per instantiation): 16
    // cost C3 8.6 % with the lights staged and 10 % without, C5 8.5 %: a
    // workgroup above ~31 KB of LDS loses a resident workgroup per CU in
    // practice (profiles/r02/ab_lds_stack.txt, profiles/r03/ab_deep_stack.txt)
    p.stack_cap = s->opt_lds_stack > 0 ? (int)s->opt_lds_stack : depth > 4 ? kLdsStackDeep : kLdsStackDefault;
    hipError_t e = launch_one(s, slot, p, maxf, mode, st, dry);
    return e == hipSuccess ? RT_OK : RT_E_HIP;
}

void free_slot(RenderSlot &r) {
    if (r.stream) (void)hipStreamSynchronize(r.stream);
    if (r.stats) (void)hipFree(r.stats);
    if (r.d_frames) (void)hipFree(r.d_frames);
    if (r.ev_in) (void)hipEventDestroy(r.ev_in);
    if (r.ev0) (void)hipEventDestroy(r.ev0);
    if (r.ev1) (void)hipEventDestroy(r.ev1);
    if (r.stream) (void)hipStreamDestroy(r.stream);
    r = RenderSlot{};
}

// own_stream: slots of a scene with more than one render in flight get a
// stream of their own, at the highest priority: HIP keeps a separate hardware
// queue pool per priority, so the slot's dispatches never queue behind barrier
// packets of caller (or collective) streams that share a hardware queue.
int init_slot(RenderSlot &r, bool own_stream) {
    if (hipMalloc(&r.stats, kStatsAlloc * sizeof(unsigned long long)) != hipSuccess) return RT_E_NOMEM;
    if (hipEventCreate(&r.ev0) != hipSuccess || hipEventCreate(&r.ev1) != hipSuccess ||
        hipEventCreateWithFlags(&r.ev_in, hipEventDisableTiming) != hipSuccess)
        return RT_E_HIP;
    if (own_stream) {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return RT_E_HIP;
        if (hipStreamCreateWithPriority(&r.stream, hipStreamNonBlocking, hi) != hipSuccess) return RT_E_HIP;
    }
    return RT_OK;
}

int set_inflight(rt_scene *s, long long n) {
    if (n < 1 || n > 8) return RT_E_INVALID;
    if ((size_t)n == s->slots.size()) return RT_OK;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    for (auto &r : s->slots) free_slot(r);
    s->slots.assign((size_t)n, RenderSlot{});
    s->next_slot = s->last_slot = 0;
    s->last_valid = false;
    for (auto &r : s->slots) {
        int rc = init_slot(r, n > 1);
        if (rc) return rc;
        // HIP binds a stream to a hardware queue at its first command: do it
        // here, not in the first frame that uses the slot
        if (r.stream && (hipMemsetAsync(r.stats, 0, sizeof(unsigned long long), r.stream) != hipSuccess ||
                         hipStreamSynchronize(r.stream) != hipSuccess))
            return RT_E_HIP;
    }
    return RT_OK;
}

// Params of one render: the scene's, with this camera and image width.
Params frame_params(const rt_scene *s, const rt_camera *cam, int W) {
    Params p = s->base;
    for (int c = 0; c < 3; c++) {
        p.eye[c] = cam->eye[c];
        p.ul[c] = cam->ul[c];
        p.dh[c] = cam->dh[c];
        p.dv[c] = cam->dv[c];
    }
    p.W = W;
    p.pix = nullptr;
    return p;
}

// Queue one render (work counter and counters reset, the launch, events) on
// the next render slot, ordered against the caller's stream `st`.
int submit(rt_scene *s, Params &p, hipStream_t st) {
    RenderSlot &slot = s->slots[(size_t)s->next_slot];
    s->last_slot = s->next_slot;
    s->next_slot = (s->next_slot + 1) % (int)s->slots.size();
    hipStream_t caller = st;
    if (slot.stream) {                 // several in flight: run on the slot's stream
        if (hipEventRecord(slot.ev_in, caller) != hipSuccess) return RT_E_HIP;
        if (hipStreamWaitEvent(slot.stream, slot.ev_in, 0) != hipSuccess) return RT_E_HIP;
        st = slot.stream;
    } else if (slot.used && hipStreamWaitEvent(st, slot.ev1, 0) != hipSuccess) {
        // one slot, any caller stream: this render reuses the slot's work
        // counter, counters and frames, so it waits for the slot's previous
        // render (issued on whatever stream) before touching them
        return RT_E_HIP;
    }
    p.stats = slot.stats;
    // one reset per frame: the counters, the work counters (kWorkSlots) and
    // the timeline (its minima are kept as maxima of the complement)
    if (hipMemsetAsync(slot.stats, 0, kStatsReset * sizeof(unsigned long long), st) != hipSuccess) return RT_E_HIP;
    (void)hipEventRecord(slot.ev0, st);
    int rc = launch(s, slot, p, st);
    (void)hipEventRecord(slot.ev1, st);
    slot.used = true;
    if (slot.stream && hipStreamWaitEvent(caller, slot.ev1, 0) != hipSuccess) return RT_E_HIP;
    s->last_valid = rc == RT_OK;
    return rc;
}

}  // namespace

extern "C" {

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *rt_strerror(int code) {
    int i = -code;
    if (i < 0 || i > 5) return "unknown error";
    return kErr[i];
}

int rt_scene_create(int device, const rt_scene_desc *desc, rt_scene **out) {
    if (!desc || !out) return RT_E_INVALID;
    *out = nullptr;
    if (desc->n_spheres < 0 || desc->n_faces < 0 || desc->n_lights < 0 || desc->n_textures < 0) return RT_E_INVALID;
    if ((desc->n_spheres && !desc->spheres) || (desc->n_faces && !desc->faces) ||
        (desc->n_lights && !desc->lights) || (desc->n_textures && !desc->textures))
        return RT_E_INVALID;
    for (int i = 0; i < desc->n_spheres; i++)
        if (desc->spheres[i].texture >= desc->n_textures) return RT_E_INVALID;
    for (int i = 0; i < desc->n_faces; i++)
        if (desc->faces[i].texture >= desc->n_textures) return RT_E_INVALID;
    for (int i = 0; i < desc->n_textures; i++)
        if (desc->textures[i].width <= 0 || desc->textures[i].height <= 0 || !desc->textures[i].rgb)
            return RT_E_INVALID;
    StepTimer tm("rt_scene_create");
    int ndev = rt_device_count();
    if (device < 0 || device >= ndev) return RT_E_NODEVICE;
    if (hipSetDevice(device) != hipSuccess) return RT_E_HIP;
    tm.mark("device");

    auto *s = new rt_scene();
    s->device = device;
    const int nf = desc->n_faces, ns = desc->n_spheres;

    // the per-object arrays and the BVH sources, on the host (rt_accel.cpp)
    accel_input(desc, s->in);
    tm.mark("host arrays");
    const AccelInput &in = s->in;
    s->secondary = in.secondary;
    std::vector<TexK> texs((size_t)desc->n_textures);

    int rc = RT_OK;
    Params &p = s->base;
    size_t tex_bytes = 0;
    for (int i = 0; i < desc->n_textures; i++) {
        const rt_texture_desc &T = desc->textures[i];
        texs[i].w = T.width, texs[i].h = T.height, texs[i].off = (long long)tex_bytes;
        tex_bytes += (size_t)T.width * T.height * 3;
    }
    // every per-object array in one device allocation, filled by one copy
    // from one host staging buffer (eight allocations and eight pageable
    // copies cost ~8 ms of a one-shot run)
    {
        Arena a;
        const size_t o_fscan = a.add(in.fscan), o_sscan = a.add(in.sscan), o_ofac = a.add(in.ofac);
        const size_t o_objs = a.add(in.objs), o_fsh = a.add(in.fsh), o_lights = a.add(in.lights);
        const size_t o_texels = a.reserve(tex_bytes), o_texs = a.add(texs);
        for (int i = 0; i < desc->n_textures; i++) {
            const rt_texture_desc &T = desc->textures[i];
            std::memcpy(a.host.data() + o_texels + (size_t)texs[i].off, T.rgb, (size_t)T.width * T.height * 3);
        }
        char *d = nullptr;
        if (hipMalloc((void **)&d, a.host.size()) != hipSuccess) {
            rc = RT_E_NOMEM;
        } else {
            s->allocs.push_back(d);
            if (hipMemcpy(d, a.host.data(), a.host.size(), hipMemcpyHostToDevice) != hipSuccess) rc = RT_E_HIP;
            p.fscan = reinterpret_cast<const float4 *>(d + o_fscan);
            p.sscan = reinterpret_cast<const float4 *>(d + o_sscan);
            p.ofac = reinterpret_cast<const float *>(d + o_ofac);
            p.objs = reinterpret_cast<const ObjK *>(d + o_objs);
            p.fsh = reinterpret_cast<const FaceShadeK *>(d + o_fsh);
            p.lights = reinterpret_cast<const LightK *>(d + o_lights);
            p.texels = reinterpret_cast<const unsigned char *>(d + o_texels);
            p.texs = reinterpret_cast<const TexK *>(d + o_texs);
        }
    }
    tm.mark("uploads");
    if (!rc && !(s->stream = take_stream(device)) &&
        hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        rc = RT_E_HIP;
    tm.mark("stream");
    if (!rc) {
        s->slots.assign(1, RenderSlot{});
        rc = init_slot(s->slots[0], false);
    }
    tm.mark("slot");
    if (!rc) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess) rc = RT_E_HIP;
        else {
            s->num_cu = prop.multiProcessorCount;
            s->max_lds = prop.sharedMemPerBlock;
        }
    }
    tm.mark("properties");
    if (rc) {
        rt_scene_destroy(s);
        return rc;
    }
    p.nf = nf;
    p.ns = ns;
    p.nl = desc->n_lights;
    for (int c = 0; c < 3; c++) p.bkg[c] = desc->bkg[c];
    p.eta_bkg = desc->eta_bkg;
    p.eps = desc->epsilon;
    p.depth = desc->depth;
    p.dir_bf = 0;                      // set with the BVH (build_bvh); the scan needs none
    p.shadow_early_out = in.nan_fac ? 0 : 1;
    // the last light's zero-Phong skip is exact when no factor is NaN (the
    // masks stay in [0, 1]) and every light colour is finite (lc * 0 = 0)
    bool lc_finite = true;
    for (const LightK &l : in.lights)
        for (float c : l.col) lc_finite = lc_finite && std::isfinite(c);
    s->last_light_skip_auto = p.shadow_early_out && lc_finite ? 1 : 0;
    p.last_light_skip = s->last_light_skip_auto;
    p.chunk = 0;                       // launch_one: chunk_for, refill_for
    p.refill_min = 1;
    p.gate_x = kGateX;
    // The origin-leaf pass for reflection and refraction rays pays in dense
    // scenes (C5: +2.3 %) and costs sparse ones (C3: -1.1 %;
    // profiles/r03/ab_origin_leaf.txt); the density is AccelInput::crossings
    // (C3: ~3, C5: ~200).
    s->crossings = in.crossings;
    s->org_first_auto = s->crossings > kOrgDensity ? kOrgFirst : 0;
    p.org_first = s->org_first_auto;
    s->lds_bytes = (size_t)(5 * nf + ns) * sizeof(float4);
    *out = s;
    return RT_OK;
}

int rt_scene_destroy(rt_scene *s) {
    if (!s) return RT_OK;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (auto &r : s->slots)           // renders still running on caller or slot streams
        if (r.ev1) (void)hipEventSynchronize(r.ev1);
    for (void *d : s->allocs) (void)hipFree(d);

    if (s->d_bvh) (void)hipFree(s->d_bvh);
    if (s->d_leafrec) (void)hipFree(s->d_leafrec);
    if (s->d_dirk) (void)hipFree(s->d_dirk);
    if (s->d_objleaf) (void)hipFree(s->d_objleaf);
    if (s->dev_out) (void)hipFree(s->dev_out);
    if (s->dev_pix) (void)hipFree(s->dev_pix);
    for (auto &r : s->slots) free_slot(r);
    if (s->stream) give_stream(s->device, s->stream);   // (synchronised above) for the next scene
    delete s;
    return RT_OK;
}

int rt_device_init(int device) {
    StepTimer tm("rt_device_init");
    const int ndev = rt_device_count();
    if (device < 0 || device >= ndev) return RT_E_NODEVICE;
    if (hipSetDevice(device) != hipSuccess || hipFree(nullptr) != hipSuccess) return RT_E_HIP;
    tm.mark("context");
    // the runtime's lazily made state: device memory, the staging paths of
    // both copy directions, a hardware queue (a stream kept for the next
    // rt_scene_create), the kernels' code object (an occupancy query)
    // (copies of 4 KB and of 1 MB: the first copy of each size class pays
    // its own staging setup -- a 33-KB counter read cost 7.5 ms after a
    // 4-KB warm-up)
    void *d = nullptr;
    std::vector<unsigned char> h((size_t)1 << 20, 0);
    int rc = RT_OK;
    if (hipMalloc(&d, h.size()) != hipSuccess) return RT_E_NOMEM;
    for (size_t n : {(size_t)4096, h.size()})
        if (hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(h.data(), d, n, hipMemcpyDeviceToHost) != hipSuccess)
            rc = RT_E_HIP;
    (void)hipFree(d);
    tm.mark("memory + copies");
    // one waiting stream per device at most: a repeated call (the API allows
    // it) adds no queue the process does not need (4 hardware queues each)
    hipStream_t st = nullptr;
    if (!rc && !pool_has(device) && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
        if (hipStreamSynchronize(st) == hipSuccess) give_stream(device, st);
        else (void)hipStreamDestroy(st);
    }
    tm.mark("stream");
    (void)render_blocks_per_cu(maxf_for_depth(4), MODE_BVH, false, 32 * 1024);
    tm.mark("code object");
    return rc;
}

int rt_scene_set_option(rt_scene *s, const char *key, long long value) {
    if (!s || !key) return RT_E_INVALID;
    std::string k(key);
    if (k == "lds") s->opt_lds = value;
    else if (k == "grid") s->opt_grid = value;
    else if (k == "reserve") s->opt_reserve = std::max(0LL, value);
    else if (k == "depth") s->base.depth = (int)value;
    else if (k == "accel") s->opt_accel = value;
    else if (k == "inflight") return set_inflight(s, value);
    else if (k == "fail_bvh_upload") s->opt_fail_bvh_upload = value;
    else if (k == "org_first") {
        if (value < -1 || value > 7) return RT_E_INVALID;
        s->base.org_first = value < 0 ? s->org_first_auto : (int)value;
    }
    else if (k == "gate_x") {
        if (value < 0 || value > 64) return RT_E_INVALID;
        s->base.gate_x = (unsigned)value;
    }
    else if (k == "refill_min") {
        if (value < 1 || value > 64) return RT_E_INVALID;
        s->opt_refill_min = value;
    }
    else if (k == "work_parts") {
        if (value != -1 && value != 1 && value != 2 && value != 4 && value != 8) return RT_E_INVALID;
        s->opt_work_parts = value;
    }
    else if (k == "chunk") {
        if (value < 0 || value > 4096) return RT_E_INVALID;
        s->opt_chunk = value;
    }
    else if (k == "lds_stack") {
        if (value < kSpill + 4 || value > kLdsStack) return RT_E_INVALID;
        s->opt_lds_stack = value;
    }
    else if (k == "bvh_presplit") {
        if (value < 0 || value > 8) return RT_E_INVALID;
        s->opt_bvh_presplit = value;
        s->bvh_D = -1.0;               // rebuild on the next render
    }
    else if (k == "bvh_leaf" || k == "bvh_collapse" || k == "bvh_node" || k == "bvh_threads") {
        if (k == "bvh_leaf") s->opt_bvh_leaf = std::max(1LL, std::min(15LL, value));
        else if (k == "bvh_collapse") s->opt_bvh_collapse = value != 0;
        else if (k == "bvh_threads") s->opt_bvh_threads = std::max(0LL, std::min(256LL, value));
        else s->opt_bvh_node = std::max(0LL, value);
        s->bvh_D = -1.0;               // rebuild on the next render
    }
    else if (k == "last_light_skip") {       // -1 auto (exact scenes), 0 off; never on where inexact
        if (value < -1 || value > 0) return RT_E_INVALID;
        s->base.last_light_skip = value < 0 ? s->last_light_skip_auto : 0;
    }
    else if (k == "counters") {
        if (value < 0 || value > 1) return RT_E_INVALID;
        s->opt_counters = value;
    }
    else if (k == "frame_share") {
        if (value != -1 && (value < 1 || value > 8)) return RT_E_INVALID;
        s->opt_frame_share = value;
    }
    else if (k == "recursive") {
        if (value < 0 || value > 1) return RT_E_INVALID;
        s->opt_recursive = value;
    }
    else return RT_E_INVALID;
    return RT_OK;
}

int rt_render_row_blocks_async(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int block, int step,
                               int nrows, float *out_rgb, void *hip_stream) {
    if (!s || !cam || !out_rgb || W < 1 || H < 1 || y0 < 0 || block < 1 || step < block || nrows < 1)
        return RT_E_INVALID;
    long long last = (long long)y0 + (long long)((nrows - 1) / block) * step + (nrows - 1) % block;
    if (last >= H) return RT_E_INVALID;
    if ((long long)W * nrows >= (1ll << 31)) return RT_E_UNSUPPORTED;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    Params p = frame_params(s, cam, W);
    p.y0 = y0;
    p.rows = nrows;
    p.rblock = block;
    p.rstep = step;
    p.total = (unsigned)((long long)W * nrows);
    p.out = out_rgb;
    return submit(s, p, hip_stream ? (hipStream_t)hip_stream : s->stream);
}

int rt_render_pixels(rt_scene *s, const rt_camera *cam, int W, int H, const int *xy, int n, float *out_rgb,
                     rt_stats *stats) {
    if (!s || !cam || !xy || !out_rgb || W < 1 || H < 1 || n < 1) return RT_E_INVALID;
    for (int k = 0; k < n; k++)
        if (xy[2 * k] < 0 || xy[2 * k] >= W || xy[2 * k + 1] < 0 || xy[2 * k + 1] >= H) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const size_t pix_bytes = (size_t)n * 2 * sizeof(int), out_bytes = (size_t)n * 3 * sizeof(float);
    // the list and the colours pass through device buffers of the scene
    if (s->dev_pix_bytes < pix_bytes) {
        if (s->dev_pix) (void)hipFree(s->dev_pix);
        s->dev_pix = nullptr;
        s->dev_pix_bytes = 0;
        if (hipMalloc(&s->dev_pix, pix_bytes) != hipSuccess) return RT_E_NOMEM;
        s->dev_pix_bytes = pix_bytes;
    }
    if (s->dev_out_bytes < out_bytes) {
        if (s->dev_out) (void)hipFree(s->dev_out);
        s->dev_out = nullptr;
        s->dev_out_bytes = 0;
        if (hipMalloc(&s->dev_out, out_bytes) != hipSuccess) return RT_E_NOMEM;
        s->dev_out_bytes = out_bytes;
    }
    // the scene's stream runs after every render issued through its slots
    for (auto &r : s->slots)
        if (r.used && hipStreamWaitEvent(s->stream, r.ev1, 0) != hipSuccess) return RT_E_HIP;
    if (hipMemcpyAsync(s->dev_pix, xy, pix_bytes, hipMemcpyHostToDevice, s->stream) != hipSuccess) return RT_E_HIP;
    Params p = frame_params(s, cam, W);
    p.y0 = 0;                          // image_row(r) = r: the list holds image rows
    p.rows = H;
    p.rblock = p.rstep = 1;
    p.total = (unsigned)n;
    p.pix = s->dev_pix;
    p.out = s->dev_out;
    int rc = submit(s, p, s->stream);
    if (rc) return rc;
    if (hipMemcpyAsync(out_rgb, s->dev_out, out_bytes, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
        hipStreamSynchronize(s->stream) != hipSuccess)
        return RT_E_HIP;
    if (stats) return rt_scene_last_stats(s, stats);
    return RT_OK;
}

static int deinterleave(const void *gathered, size_t elem_bytes, int world, int rows_per, int W, int H, int block,
                        void *image, void *hip_stream) {
    if (!gathered || !image || world < 1 || rows_per < 1 || W < 1 || H < 1 || block < 1) return RT_E_INVALID;
    // every image row's source row must exist: each rank's row count <= rows_per
    const int nblocks = (H + block - 1) / block;
    for (int r = 0; r < world; r++) {
        int rows = 0;
        for (int b = r; b < nblocks; b += world) rows += std::min(block, H - b * block);
        if (rows > rows_per) return RT_E_INVALID;
    }
    return deinterleave_launch(gathered, (size_t)W * 3 * elem_bytes, elem_bytes, world, rows_per, H, block, image,
                               (hipStream_t)hip_stream) == hipSuccess
               ? RT_OK
               : RT_E_HIP;
}

int rt_deinterleave_rows(const float *gathered, int world, int rows_per, int W, int H, int block, float *image,
                         void *hip_stream) {
    return deinterleave(gathered, sizeof(float), world, rows_per, W, H, block, image, hip_stream);
}

int rt_deinterleave_rows_u8(const unsigned char *gathered, int world, int rows_per, int W, int H, int block,
                            unsigned char *image, void *hip_stream) {
    return deinterleave(gathered, 1, world, rows_per, W, H, block, image, hip_stream);
}

int rt_quantize_u8(const float *rgb, long long n, unsigned char *out, unsigned *flag, void *hip_stream) {
    if (!rgb || !out || !flag || n < 0) return RT_E_INVALID;
    if ((reinterpret_cast<uintptr_t>(rgb) & 15) || (reinterpret_cast<uintptr_t>(out) & 3)) return RT_E_INVALID;
    return quantize_u8_launch(rgb, (size_t)n, out, flag, (hipStream_t)hip_stream) == hipSuccess ? RT_OK : RT_E_HIP;
}

int rt_scene_prepare(rt_scene *s, const rt_camera *cam, int W, int H) {
    if (!s || !cam || W < 1 || H < 1) return RT_E_INVALID;
    if ((long long)W * H >= (1ll << 31)) return RT_E_UNSUPPORTED;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    Params p = s->base;
    for (int c = 0; c < 3; c++) {
        p.eye[c] = cam->eye[c];
        p.ul[c] = cam->ul[c];
        p.dh[c] = cam->dh[c];
        p.dv[c] = cam->dv[c];
    }
    p.W = W;
    p.rows = H;
    p.total = (unsigned)((long long)W * H);
    int rc = launch(s, s->slots[0], p, s->stream, true);
    if (rc == RT_OK && hipDeviceSynchronize() != hipSuccess) rc = RT_E_HIP;
    return rc;
}

int rt_render_rows_async(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int y1, float *out_rgb,
                         void *hip_stream) {
    if (y1 <= y0) return RT_E_INVALID;
    return rt_render_row_blocks_async(s, cam, W, H, y0, y1 - y0, y1 - y0, y1 - y0, out_rgb, hip_stream);
}

// The last render's counters with the exit counters' copies folded in
// (rt_device.h kStatCopies).
static hipError_t read_counters(const RenderSlot &slot, unsigned long long h[kNStats]) {
    std::vector<unsigned long long> all(kStatsReset);
    hipError_t e = hipMemcpy(all.data(), slot.stats, all.size() * sizeof(all[0]), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    std::memcpy(h, all.data(), kNStats * sizeof(h[0]));
    static const int kAdd[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 32, 33, 34};
    for (int c = 0; c < kStatCopies; c++) {
        const unsigned long long *sc = all.data() + stat_copy_off(c);
        for (int k : kAdd) h[k] += sc[k];
        h[24] = std::max(h[24], sc[24]);
        h[26] = std::max(h[26], sc[26]);
    }
    return hipSuccess;
}

int rt_scene_last_stats(rt_scene *s, rt_stats *stats) {
    if (!s || !stats) return RT_E_INVALID;
    if (!s->last_valid) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const RenderSlot &slot = s->slots[(size_t)s->last_slot];
    if (hipEventSynchronize(slot.ev1) != hipSuccess) return RT_E_HIP;
    unsigned long long h[kNStats];
    if (read_counters(slot, h) != hipSuccess) return RT_E_HIP;
    stats->primary = h[0];
    stats->shadow = h[1];
    stats->refraction = h[2];
    stats->reflection = h[3];
    stats->skip_trans = h[4];
    stats->ub_back = h[5];
    stats->box_tests = h[6];
    stats->face_tests = h[7];
    stats->sphere_tests = h[8];
    stats->shadow_known = h[32];
    stats->bf_queries = h[33];
    stats->stack_spills = h[34];
    stats->bvh_build_ms = s->bvh_build_ms;
    // device time of the launch: first wave start .. last wave end (100 MHz
    // clock); the events' interval also holds any wait for a previous frame
    // still on the CUs
    const unsigned long long t0 = ~h[24];          // the first wave's start (stored complemented)
    if (h[24] != 0 && h[26] > t0) {
        stats->kernel_ms = (double)(h[26] - t0) * 1e-5;
    } else {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, slot.ev0, slot.ev1);
        stats->kernel_ms = ms;
    }
    return RT_OK;
}

int rt_scene_debug_counters(rt_scene *s, unsigned long long *out, int n) {
    if (!s || !out || n < 0 || n > kNStats || !s->last_valid) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const RenderSlot &slot = s->slots[(size_t)s->last_slot];
    if (hipEventSynchronize(slot.ev1) != hipSuccess) return RT_E_HIP;
    unsigned long long h[kNStats];
    if (read_counters(slot, h) != hipSuccess) return RT_E_HIP;
    // minima kept complemented on the device (one memset per frame)
    for (int k = 24; k <= 25; k++) h[k] = h[k] ? ~h[k] : ~0ull;
    h[16] = (unsigned long long)s->last_mode;
    h[17] = (unsigned long long)s->last_blocks_per_cu;
    h[18] = (unsigned long long)s->last_grid;
    h[19] = (unsigned long long)s->last_lds;
    h[20] = (unsigned long long)s->bvh_nodes;
    h[21] = (unsigned long long)s->bvh_depth;
    h[22] = (unsigned long long)s->bvh_stack;
    h[23] = (unsigned long long)s->num_cu;
    h[40] = (unsigned long long)s->last_org_first;
    h[41] = (unsigned long long)(s->crossings * 1000.0);
    h[42] = (unsigned long long)s->last_stack_cap;
    h[43] = (unsigned long long)s->last_lights_in_lds;
    h[45] = (unsigned long long)s->last_work_parts;
    h[44] = 0;                                   // (round 4-5: the BVH top copies, option removed)
    h[46] = (unsigned long long)s->last_maxf;
    h[47] = head_split((int)s->last_maxf) ? 1 : 0;
    h[48] = (unsigned long long)s->opt_counters;
    for (int i = 0; i < n; i++) out[i] = h[i];
    return RT_OK;
}

int rt_scene_debug_ub_pixels(rt_scene *s, int *xy, int n) {
    if (!s || (n > 0 && !xy) || n < 0 || !s->last_valid) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const RenderSlot &slot = s->slots[(size_t)s->last_slot];
    if (hipEventSynchronize(slot.ev1) != hipSuccess) return RT_E_HIP;
    unsigned long long events = 0;
    if (hipMemcpy(&events, slot.stats + 44, sizeof events, hipMemcpyDeviceToHost) != hipSuccess) return RT_E_HIP;
    const size_t k = (size_t)std::min<unsigned long long>({events, (unsigned long long)kUbLogMax,
                                                            (unsigned long long)n});
    std::vector<unsigned long long> v(k);
    if (k > 0 && hipMemcpy(v.data(), slot.stats + kUbLogOff, k * sizeof v[0], hipMemcpyDeviceToHost) != hipSuccess)
        return RT_E_HIP;
    for (size_t i = 0; i < k; i++) xy[2 * i] = (int)(v[i] >> 32), xy[2 * i + 1] = (int)(unsigned)v[i];
    return (int)std::min<unsigned long long>(events, (unsigned long long)INT32_MAX);
}

int rt_scene_debug_wavelog(rt_scene *s, unsigned long long *out, int n) {
    if (kWaveLogMax == 0) return RT_E_INVALID;   // not an RT_PROF build
    if (!s || !out || n < 0 || !s->last_valid) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const RenderSlot &slot = s->slots[(size_t)s->last_slot];
    if (hipEventSynchronize(slot.ev1) != hipSuccess) return RT_E_HIP;
    const long long waves = std::min<long long>(s->last_grid * (kBlock / 64), kWaveLogMax);
    const int words = (int)std::min<long long>(n, waves * kWaveLogWords);
    if (words > 0 && hipMemcpy(out, slot.stats + kWaveLogOff, (size_t)words * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost) != hipSuccess)
        return RT_E_HIP;
    return words;
}

int rt_render_rows(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int y1, float *out_rgb, rt_stats *stats) {
    if (!s || !cam || !out_rgb || W < 1 || H < 1 || y0 < 0 || y1 > H || y0 >= y1) return RT_E_INVALID;
    return rt_render_row_blocks(s, cam, W, H, y0, y1 - y0, y1 - y0, y1 - y0, out_rgb, stats);
}

int rt_render_row_blocks(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int block, int step, int nrows,
                         float *out_rgb, rt_stats *stats) {
    if (!s || !cam || !out_rgb || nrows < 1) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    hipPointerAttribute_t attr;
    bool on_device = false;
    if (hipPointerGetAttributes(&attr, out_rgb) == hipSuccess)
        on_device = attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
    else
        (void)hipGetLastError();
    size_t bytes = (size_t)W * (size_t)nrows * 3 * sizeof(float);
    float *dst = out_rgb;
    if (!on_device) {
        if (s->dev_out_bytes < bytes) {
            if (s->dev_out) (void)hipFree(s->dev_out);
            s->dev_out = nullptr;
            s->dev_out_bytes = 0;
            if (hipMalloc(&s->dev_out, bytes) != hipSuccess) return RT_E_NOMEM;
            s->dev_out_bytes = bytes;
        }
        dst = s->dev_out;
    }
    StepTimer tm("rt_render_row_blocks");
    int rc = rt_render_row_blocks_async(s, cam, W, H, y0, block, step, nrows, dst, nullptr);
    if (rc) return rc;
    tm.mark("submitted");
    if (!on_device && hipMemcpyAsync(out_rgb, dst, bytes, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
        return RT_E_HIP;
    if (hipStreamSynchronize(s->stream) != hipSuccess) return RT_E_HIP;
    tm.mark("synchronized");
    if (stats) rc = rt_scene_last_stats(s, stats);
    tm.mark("stats");
    return rc;
}

}  // extern "C"