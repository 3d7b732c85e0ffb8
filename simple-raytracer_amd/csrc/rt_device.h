// rt_device.h -- what the render kernel (rt_kernels.hip) and the host side
// (rt_scene.cpp: scene upload, render slots, the rt_hip.h C ABI) share: the
// float semantics of the reference's Vector3 / Color (src/definitions.h:18-195),
// the device scene layout (Params and its arrays), and the
// launch interface of the kernels.  Internal to librt_hip.so.
#ifndef RT_DEVICE_H
#define RT_DEVICE_H

#include <hip/hip_runtime.h>

#include <cstddef>

namespace rt {

// ---------------------------------------------------------------------------
// Device-side geometry/colour semantics of src/definitions.h
// ---------------------------------------------------------------------------
struct V3 {
    float x, y, z;
};
struct C3 {
    float r, g, b;
};

__host__ __device__ __forceinline__ V3 vadd(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__host__ __device__ __forceinline__ V3 vsub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__host__ __device__ __forceinline__ V3 vmul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__host__ __device__ __forceinline__ V3 vdiv(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__host__ __device__ __forceinline__ float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ V3 vnorm(V3 a) { return vdiv(a, sqrtf(vdot(a, a))); }
__host__ __device__ __forceinline__ V3 vcross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// std::clamp(v, 0, 1): NaN passes through (not fminf/fmaxf).  Through the
// NaN-propagating IEEE maximum / minimum (gfx950 v_maximum3_f32 /
// v_minimum3_f32): two instructions instead of two compares and two selects;
// the one difference from std::clamp is -0 -> +0, a sign of zero no later
// colour operation distinguishes (relaxation 6)
__device__ __forceinline__ float clamp01(float v) {
    return __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, 0.0f), 1.0f);
}
__device__ __forceinline__ float clampr(float v, float lo, float hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }
__device__ __forceinline__ C3 cmulc(C3 a, C3 b) { return {clamp01(b.r * a.r), clamp01(b.g * a.g), clamp01(b.b * a.b)}; }
__device__ __forceinline__ C3 cmulf(C3 a, float f) { return {clamp01(f * a.r), clamp01(f * a.g), clamp01(f * a.b)}; }
__device__ __forceinline__ C3 cadd(C3 a, C3 b) { return {clamp01(b.r + a.r), clamp01(b.g + a.g), clamp01(b.b + a.b)}; }
__device__ __forceinline__ float max0(float x) { return (0.0f < x) ? x : 0.0f; }

constexpr double kPi = 3.14159265358979323846;        // src/config.h:11
constexpr double kRightAngle = 90.0 * kPi / 180.0;    // main.cpp:964
constexpr float kFltMax = 3.40282347e+38f;            // std::numeric_limits<float>::max()

enum { ENTERING = 0, EXITING = 1 };

// ---------------------------------------------------------------------------
// Device scene layout (built by rt_scene_create)
// ---------------------------------------------------------------------------
// Faces (object index 0..nf-1), 5 x float4 each, per-face invariants hoisted
// exactly as TraceRay computes them (main.cpp:1280-1301, :1361-1366):
//   [0] v0.xyz, D = -n.v0     [1] n.xyz, det = d11*d22 - d12*d12
//   [2] e1.xyz, d11           [3] e2.xyz, d22        [4] d12, -, -, -
// Spheres (object index nf..nf+ns-1): float4 center.xyz, radius.
struct ObjK {                 // per object, shading data
    float dif[3], ka;
    float spc[3], kd;
    float ks, n, opacity, eta;
    int tex;                  // texture index or -1
    int is_sphere;
    int pad[2];
};
struct FaceShadeK {           // per face, shading-only data
    float vn[3][3];           // vertex_normal[k].norm() (main.cpp:1382-1384)
    float vt[3][2];           // clamp<float>(texture_coords, 0, 1) (main.cpp:835-841)
    int smooth;
    int pad[2];
};
struct LightK {
    float xyz[3], w;          // position or direction, w
    float col[3], pad0;
    float L[3], pad1;         // directional: light.direction.norm() * -1 (main.cpp:887)
    float sdir[3], pad2;      // directional: light.direction * -1 (main.cpp:895, unnormalised)
};
static_assert(sizeof(LightK) % sizeof(float4) == 0, "lights are staged in LDS as float4s");
struct TexK {
    int w, h;
    long long off;                       // first byte in Params::texels
};
// directional light: its shadow-region tree over the spheres (rt host:
// dir_trees) -- root node in Params::bvh (-1: no sphere can shadow) and the
// rotation R (rows) into the frame the tree's boxes were built in
struct DirK {
    float R[9];
    int root;
    float cone_k;                        // max(0, |d|^2 - 1), rounded up
    float cone_h;                        // |d| < 1: height bound of the shadow region, else +inf
};

struct Params {
    const float4 *__restrict__ fscan;
    const float4 *__restrict__ sscan;
    const float *__restrict__ ofac;      // (float)(1.0 - opacity) per object (main.cpp:909)
    const ObjK *__restrict__ objs;
    const FaceShadeK *__restrict__ fsh;
    const LightK *__restrict__ lights;
    const unsigned char *__restrict__ texels;   // all textures: RGB bytes, row-major
    const TexK *__restrict__ texs;
    float *__restrict__ out;
    unsigned long long *__restrict__ stats;
    int nf, ns, nl;
    float bkg[3];
    float eta_bkg, eps;
    int depth;
    float eye[3], ul[3], dh[3], dv[3];
    int W, y0, rows;                     // render `rows` rows of a W-wide image: local row r is
    int rblock, rstep;                   // image row y0 + (r / rblock) * rstep + r % rblock
    unsigned int total;                  // W * rows, or the pixel list's length
    // BVH (MODE_BVH): 8 float4 per 4-wide node (rt_bvh.h Node4), leaf-ordered object keys
    const float4 *__restrict__ bvh;
    int last_light_skip;                 // a last light with a Phong sum of 0 is not searched (advance)
    const float4 *__restrict__ leafrec;  // leaf-ordered primitive records (rt_bvh.h leaf_records)
    int dir_bf;                          // directional lights in a scene with spheres: 0 none,
                                         // 1 brute-force scan, 2 faces by the BVH + shadow-region trees
    const DirK *__restrict__ dirk;       // per light (dir_bf == 2)
    int shadow_early_out;                // no NaN shadow factor: an opaque hit ends a shadow ray
    int ovf_stride;                      // BVH: stack spill entries per lane (deepest tree, kSpill multiple)
    int lights_lds;                      // the lights' copy in LDS: float4 offset in rt_lds
    int stack_cap;                       // BVH: stack entries kept in LDS (<= kLdsStack)
    unsigned chunk;                      // work items a wave takes from the counter at a time (0: its idle lanes' count)
    unsigned refill_min;                 // refill only when at least this many lanes are idle (or all are)
    unsigned gate_x;                     // hold reflection/refraction searches until this many lanes have one
    unsigned work_shift;                 // 2^work_shift work item bands with a counter each (3: one per XCD)
    void *__restrict__ frames;           // grid x kBlock x MAXF cold ShadeRay frames
    int *__restrict__ ovf;               // grid x kBlock x ovf_stride spilled BVH stack entries
    const int *__restrict__ pix;         // pixel list (x, y pairs; rt_render_pixels) or null: work item k
                                         // is pixel (pix[2k], pix[2k+1]), its colour goes to out[3k..3k+2]
    int lights_in_lds;                   // 1: the lights are staged in LDS; 0: read from `lights` (too many)
    const int *__restrict__ objleaf;     // BVH: per object, the link of its leaf in the main tree
    int org_first;                       // origin-leaf pass: bit 0 shadow, 1 refraction, 2 reflection rays
    void *heads;                         // dense frame heads (dense_heads(MAXF)): [block][level][lane] 32-B slots
};

enum Mode { MODE_SCAN = 0, MODE_SCAN_LDS = 1, MODE_BVH = 2 };
#ifndef RT_PROF
#define RT_PROF 0                        // 1: per-wave cycle/occupancy counters in stats[9..15]
#endif
#ifndef RT_PRIO
#define RT_PRIO 1                        // 1: shading steps at wave priority 2 (render_kernel)
#endif
#ifndef RT_CHECK
#define RT_CHECK 0                       // 1: check the BVH stack-bottom invariant (lib_check/, never benched):
                                         // violations counted in stats[kCheckSlot]
#endif
constexpr int kCheckSlot = 49;
#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 5                   // waves per SIMD the register budget must allow (A/B: 5 best)
#endif
// Largest worst-case BVH stack a tree may need (entries per lane; the spill
// area is sized per tree, Params::ovf_stride).  Refill tags kRefill + b stay
// far below the leaf links (> INT_MIN + 256) for b <= kStackMax / kSpill.
constexpr int kStackMax = 512;
// BVH traversal stack entries per lane in LDS (entry 0: the sentinel); a
// deeper stack spills its oldest kSpill entries to device memory (rare)
constexpr int kLdsStack = 16;            // most entries the LDS share may hold (option lds_stack)
#ifndef RT_LDS_STACK
#define RT_LDS_STACK 15                  // 16 (32 KB per block with the shading state): 5 blocks per CU
                                         // on paper, -8.6 % measured; 15 (31.8 KB): C3 +-0, C4 +0.5 %
                                         // against 14 (profiles/r05/ab/lds_stack15_*.txt)
#endif
constexpr int kLdsStackDefault = RT_LDS_STACK;
#ifndef RT_LDS_STACK_DEEP
#define RT_LDS_STACK_DEEP 15             // depth > 4 (render_kernel<9 / 17, *>): 16 entries with the
                                         // lights in device memory (32 KB per block) cost C5 8.5 %
                                         // (profiles/r03/ab_deep_stack.txt), 15 gains 0.55 % on C5 (r05)
#endif
constexpr int kLdsStackDeep = RT_LDS_STACK_DEEP;
#ifndef RT_SPILL
#define RT_SPILL 8
#endif
constexpr int kSpill = RT_SPILL;
static_assert(kStackMax % kSpill == 0 && kStackMax / kSpill < 200 && kLdsStack - 3 > kSpill, "stack spill blocks");
#ifndef RT_BLOCK
#define RT_BLOCK 256                     // lanes per workgroup of render_kernel
#endif
constexpr int kBlock = RT_BLOCK;
constexpr long long kCounters = 1;       // option counters default (the instantiation without is ~4 % faster)
#ifndef RT_FRAME_SHARE
#define RT_FRAME_SHARE 2                 // option frame_share's automatic value for small frames in flight
#endif
constexpr long long kFrameShare = RT_FRAME_SHARE;
#ifndef RT_FRAME_SHARE_ITEMS
#define RT_FRAME_SHARE_ITEMS 32          // ... for frames of at most this many work items per lane of the grid
#endif
constexpr unsigned long long kFrameShareItems = RT_FRAME_SHARE_ITEMS;
// every recursive instantiation keeps its frame heads in dense [block][level]
// [lane] arrays (rt_kernels.hip Fr; MAXF 1 opens no child)
constexpr bool dense_heads(int maxf) { return maxf > 1; }
// The dense frame slots of an instantiation with MAXF <= 9 are split: 16-B
// colour heads and 16-B stack slots in two arrays, the node's meta carrying a
// bit per level instead (rt_kernels.hip Fr, kKindsShift); MAXF 17 keeps one
// 32-B slot per level (acc, f, meta, 3 stack entries).  32 B per slot either way.
constexpr bool head_split(int maxf) { return dense_heads(maxf) && maxf <= 9; }
constexpr int kSplitLightBits = 15;      // light index bits of a head_split instantiation's meta
constexpr int kSplitLightMax = (1 << kSplitLightBits) - 1;   // more lights: MAXF 17 (rt_scene.cpp)
constexpr int head_stack(int maxf) { return head_split(maxf) ? 4 : 3; }   // medium-stack entries in a dense slot
constexpr int kHeadInts = 8;             // 4-B words per dense slot (a 64-B slot: C5 -1.7 %, profiles/r06/heads)
constexpr unsigned kGateX = 32;          // option gate_x (A/B: 24..48 within 0.2 % on C3 and C5)
#ifndef RT_ORG_FIRST
#define RT_ORG_FIRST 6                   // option org_first: origin-leaf pass for shadow (1) / refraction (2) /
                                         // reflection (4) rays -- in scenes denser than kOrgDensity
#endif
constexpr int kOrgFirst = RT_ORG_FIRST;
constexpr double kOrgDensity = 32.0;     // objects met by a line across the scene (C3 ~3, C5 ~200)
constexpr int kNStats = 64;              // counter slots (rt_scene_debug_counters; the device writes 0..39, 44)
// RT_PROF builds: a per-wave timeline after the counters (rt_scene_debug_wavelog),
// kWaveLogWords words per wave: launch start, prologue done, work drained (0:
// never saw it), end (100 MHz ticks), HW_ID, XCC_ID, outer iterations, refills
#if RT_PROF
constexpr int kWaveLogWords = 8;
constexpr int kWaveLogMax = 16384;       // waves (grid x kBlock / 64 <= 1280 x 4 on MI355X)
#else
constexpr int kWaveLogWords = 8;
constexpr int kWaveLogMax = 0;
#endif
// Pixel work counters after the counters: one per band of the work items
// (2^Params::work_shift bands, one per XCD: workgroup b runs on XCD b mod 8),
// each a 32-bit counter 4 KB from the next (device-scope atomics are done
// memory-side: counters on one channel would queue behind each other); the
// one memset before a render (kStatsReset slots) resets them with the counters.
constexpr int kWorkSlots = kNStats;      // band b's counter: u64 slot kWorkSlots + kWorkStride * b
constexpr int kWorkStride = 512;
constexpr int kWorkPartsMax = 8;
constexpr int kStatsReset = kWorkSlots + kWorkStride * kWorkPartsMax;
// The exit-time counters of every wave ([0..8], [24], [26], [32..34]) go to
// kStatCopies copies of the counter array, copy c in the free words of band
// (c mod 8)'s counter block, 512 B or 1.5 KB past the counter: thousands of
// waves ending within microseconds of each other, each adding to the same
// few words, queued behind each other in one memory channel.  The host folds
// the copies (sum; maximum for [24] and [26]).
constexpr int kStatCopies = 16;
constexpr int stat_copy_off(int c) { return kWorkSlots + kWorkStride * (c & 7) + 64 + (c >> 3) * 128; }
static_assert(64 + 128 + kNStats <= kWorkStride, "stat copies fit a band's counter block");
// Pixels whose shade tree read back() of an empty medium stack (main.cpp:1028,
// UB in the reference): stats[44] counts the events, the first kUbLogMax
// pixels follow the work counters as x << 32 | y (rt_scene_debug_ub_pixels)
constexpr int kUbLogOff = kStatsReset;
constexpr int kUbLogMax = 4096;
constexpr int kWaveLogOff = kUbLogOff + kUbLogMax;
constexpr int kStatsAlloc = kWaveLogOff + kWaveLogWords * kWaveLogMax;
constexpr int kLdsHotWords = 16;         // per-lane shading state words in LDS (rt_kernels.hip LW_*)

// ---------------------------------------------------------------------------
// Launch interface (rt_kernels.hip)
// ---------------------------------------------------------------------------
// MAXF, the ShadeRay frames per lane an instantiation holds, for a recursion
// depth: 5 (depth <= 4), 9 (<= 8), 17 (<= 16); -1 above
int maxf_for_depth(int depth);
// the instantiation for a scene: 1 when no material reflects or refracts (or
// depth 0), else by depth (-1: deeper than supported)
int maxf_for(int depth, bool secondary);
// resident workgroups per CU of render_kernel<maxf, mode, count> with
// `lds_bytes` of dynamic LDS (0 if it cannot launch)
int render_blocks_per_cu(int maxf, int mode, bool count, size_t lds_bytes);
// bytes of one lane's cold ShadeRay frame (Cold<maxf>)
size_t cold_frame_bytes(int maxf);
// rt_quantize_u8 (rgb: n floats, 16-B aligned; out: n bytes, 4-B aligned)
hipError_t quantize_u8_launch(const float *rgb, size_t n, unsigned char *out, unsigned *flag, hipStream_t st);
// count: the instantiation with the counters (rays by kind, events, executed
// tests; option counters; rt_kernels.hip RT_COUNT)
hipError_t render_launch(int maxf, int mode, bool count, const Params &p, unsigned grid, size_t lds_bytes,
                         hipStream_t st);
// gathered row sets -> image order; a row is row_bytes bytes of elements of
// elem_bytes (4: floats, 1: the writer's bytes)
hipError_t deinterleave_launch(const void *gathered, size_t row_bytes, size_t elem_bytes, int world, int rows_per,
                               int H, int block, void *image, hipStream_t st);

}  // namespace rt

#endif  // RT_DEVICE_H
