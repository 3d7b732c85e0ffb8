/*
 * rt_hip.h -- C ABI of the MI355X (gfx950) ray-trace layer.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * has no plugin API; its seam is the single call
 *
 *     Mat3D create_view_window_and_ray_trace(eye, viewdir.norm(), updir.norm(),
 *                                            fov_h, height, width, bkg);
 *         -- /root/reference/main.cpp:607 (definition :670-767)
 *
 * plus the implicit inputs it reads from the global `Globals environment`
 * (main.cpp:58, type src/definitions.h:304-311): spheres, faces, lights,
 * materials, textures, "epsilon", "recursion_depth", "bkg_refraction_index".
 * Under it run TraceRay (main.cpp:1215-1407) and ShadeRay (main.cpp:783-1207).
 *
 * Here that seam is split into: an explicit, POD scene description
 * (rt_scene_desc: what `environment` held), a per-image camera (rt_camera:
 * main.cpp:677-710, computed on the host by rt_host.h's rth_camera) and a
 * row-range render (rt_render_rows: the pixel loop main.cpp:718-764 and
 * everything below it) returning pre-quantisation float RGB.  Quantisation
 * to the reference's size_t pixels (main.cpp:760-762) and the P3 writer
 * (main.cpp:613-650) live in rt_host.h.
 *
 * Conventions: plain C, no exceptions cross the ABI, every function returns
 * RT_OK (0) or a negative RT_E_* code (rt_strerror gives the text).  The
 * caller owns every buffer it passes; the library keeps device copies inside
 * rt_scene and never retains caller pointers after a call returns.
 * rt_scene objects are per device; distinct scenes may be used from
 * different host threads concurrently.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_E_INVALID (-1)     /* bad argument / malformed description */
#define RT_E_NODEVICE (-2)    /* no such HIP device */
#define RT_E_HIP (-3)         /* a HIP runtime call failed */
#define RT_E_NOMEM (-4)       /* device allocation failed */
#define RT_E_UNSUPPORTED (-5) /* e.g. recursion depth above the compiled maximum */

/* Material (src/definitions.h:249-253, parsed at main.cpp:272-308). */
typedef struct {
    float diffuse[3];
    float specular[3];
    float ka, kd, ks, n;
    float opacity;       /* already clamped to [0,1] by the parser (main.cpp:294) */
    float eta;           /* refraction index */
} rt_material;

/* 'sphere' (main.cpp:328-377). texture = index into textures, or -1. */
typedef struct {
    float center[3];
    float radius;
    rt_material mat;
    int texture;
} rt_sphere_desc;

/* 'f' (main.cpp:470-552).  v/vn/vt are the resolved vertex data (missing
 * indices resolve to zero, like the reference's std::map::operator[]).
 * smooth = the reference's smooth_shading flag (decided by the LAST vertex
 * token's format). */
typedef struct {
    float v[3][3];
    float vn[3][3];
    float vt[3][2];
    int smooth;
    rt_material mat;
    int texture;
} rt_face_desc;

/* 'light x y z w r g b' (main.cpp:378-411): w == 0 -> directional (xyz is the
 * direction), else point (xyz is the position). */
typedef struct {
    float xyz[3];
    float w;
    float color[3];
} rt_light_desc;

/* P3 texture (src/utility.h:59-139): rgb is [height][width][3] bytes. */
typedef struct {
    int width, height;
    const unsigned char *rgb;
} rt_texture_desc;

/* Everything the reference kept in `environment` for the hot path.  Objects
 * are given per type in FILE order; the renderer visits all faces before all
 * spheres, as the reference's std::map<string,...> iteration does
 * (main.cpp:1218). */
typedef struct {
    int n_spheres;
    const rt_sphere_desc *spheres;
    int n_faces;
    const rt_face_desc *faces;
    int n_lights;
    const rt_light_desc *lights;
    int n_textures;
    const rt_texture_desc *textures;
    float bkg[3];        /* bkgcolor r g b */
    float eta_bkg;       /* bkgcolor 4th arg; 0 when absent (main.cpp:751 default-insert) */
    float epsilon;       /* 1e-3 (main.cpp:101) */
    int depth;           /* recursion depth, 4 in the reference (main.cpp:100) */
} rt_scene_desc;

/* Per-image constants of main.cpp:677-710: pixel (i, j) looks along
 * ((ul + dh*j) + dv*i) - eye. */
typedef struct {
    float eye[3];
    float ul[3];
    float dh[3];
    float dv[3];
} rt_camera;

/* Ray counters.  One ray = one TraceRay call of the reference. */
typedef struct {
    unsigned long long primary;
    unsigned long long shadow;
    unsigned long long refraction;
    unsigned long long reflection;
    unsigned long long skip_trans;   /* 'goto SKIP_TRANS' taken (main.cpp:1001) */
    unsigned long long ub_back;      /* back() on an empty medium stack (main.cpp:1028, UB in the reference) */
    double kernel_ms;                /* device time of the render kernel(s) */
    unsigned long long box_tests;    /* ray-box tests executed (BVH traversal) */
    unsigned long long face_tests;   /* ray-triangle tests executed */
    unsigned long long sphere_tests; /* ray-sphere tests executed */
    unsigned long long shadow_known; /* shadow rays counted above whose cumulative mask was already 0:
                                        their result is known, they are not searched */
    unsigned long long bf_queries;   /* queries answered by the brute-force scan (BVH mode fallbacks) */
    unsigned long long stack_spills; /* BVH traversal stack blocks spilled from LDS to device memory */
    double bvh_build_ms;             /* host time of the scene's last BVH (re)build (0: none) */
} rt_stats;

typedef struct rt_scene rt_scene;

int rt_device_count(void);

/* Optional: start the HIP runtime and the state it makes lazily on first use
 * for `device` -- the context, device memory, the copy paths, a hardware queue
 * (a stream the next rt_scene_create on the device takes), the kernels' code
 * object -- ahead of rt_scene_create, e.g. on a thread while the scene file
 * is parsed (the CLI does: ~40-50 ms that would otherwise land in the first
 * scene upload and the first stats read).  Thread-safe; may be called again:
 * at most one such stream waits per device (a repeated call adds none). */
int rt_device_init(int device);

/* Upload a scene to HIP device `device`. */
int rt_scene_create(int device, const rt_scene_desc *desc, rt_scene **out);
int rt_scene_destroy(rt_scene *scene);

/* Render image rows [y0, y1) of a W x H image into out_rgb, which holds
 * (y1 - y0) * W * 3 floats (row-major, RGB) and may be host or device
 * memory.  Synchronous.  stats may be NULL.  W, H >= 1: the seam itself
 * (main.cpp:670) takes any size -- a 1-pixel-wide or -tall image divides by
 * res - 1 = 0 (main.cpp:709-710), its camera deltas are NaN / inf
 * (rth_camera does the same), every primary ray is NaN and meets nothing, and
 * every pixel is the background, as in the reference.  (The reference's
 * parser rejects such an imsize before the seam, main.cpp:242; so does
 * rt_host.h's.) */
int rt_render_rows(rt_scene *scene, const rt_camera *cam, int W, int H, int y0, int y1, float *out_rgb,
                   rt_stats *stats);

/* Same, asynchronous on `hip_stream` (a hipStream_t, NULL = the scene's own
 * stream); out_rgb must be device memory.  The render is ordered after the
 * work already queued on hip_stream and before the work queued after it.
 * rt_scene_last_stats() waits for the last render and returns its counters
 * (kernel_ms = first wave start .. last wave end of its launch). */
int rt_render_rows_async(rt_scene *scene, const rt_camera *cam, int W, int H, int y0, int y1, float *out_rgb,
                         void *hip_stream);
int rt_scene_last_stats(rt_scene *scene, rt_stats *stats);

/* Block-interleaved row set, asynchronous (device out_rgb): local row r
 * (0 <= r < nrows) is image row y0 + (r / block) * step + r % block, written
 * to out_rgb row r.  With y0 = 8*rank, block = 8, step = 8*N the N ranks of a
 * multi-GPU render get equally mixed rows (load balance). */
int rt_render_row_blocks_async(rt_scene *scene, const rt_camera *cam, int W, int H, int y0, int block, int step,
                               int nrows, float *out_rgb, void *hip_stream);

/* Optional: build the acceleration structure for this camera and size every
 * render slot's buffers for a W x H image now, so that no later render pays
 * for either (the first render would, once).  Renders nothing. */
int rt_scene_prepare(rt_scene *scene, const rt_camera *cam, int W, int H);

/* Synchronous form of rt_render_row_blocks_async: out_rgb (nrows * W * 3
 * floats) may be host or device memory.  stats may be NULL. */
int rt_render_row_blocks(rt_scene *scene, const rt_camera *cam, int W, int H, int y0, int block, int step,
                         int nrows, float *out_rgb, rt_stats *stats);

/* Render a list of n pixels of the W x H image: xy holds n (x, y) pairs
 * (host memory), out_rgb receives n * 3 floats (host memory), pixel k's
 * colour at out_rgb[3k..3k+2] -- bit for bit the colour the whole-image
 * render gives that pixel; stats count the list's rays only.  Synchronous,
 * on the scene's stream after every render issued before.  (Sparse
 * re-renders; the parity tests use it for exact per-pixel ray counts on
 * samples of full-size images.)  stats may be NULL. */
int rt_render_pixels(rt_scene *scene, const rt_camera *cam, int W, int H, const int *xy, int n, float *out_rgb,
                     rt_stats *stats);

/* Put gathered row sets back in image order, on the device (the multi-device
 * CLI: after an RCCL gather of every device's rt_render_row_blocks buffer).
 * gathered holds `world` buffers of rows_per * W * 3 floats, buffer r being
 * rank r's rows as rth_row_set deals them (blocks of `block` rows, round
 * robin); image receives H * W * 3 floats.  Both are device memory of the
 * current device; asynchronous on hip_stream. */
int rt_deinterleave_rows(const float *gathered, int world, int rows_per, int W, int H, int block, float *image,
                         void *hip_stream);
/* The same for the writer's values as bytes (rt_quantize_u8 output, 3 per
 * pixel): one kernel puts a byte gather of N ranks in image order (bench.py
 * rank 0 at N > 1, instead of N index copies). */
int rt_deinterleave_rows_u8(const unsigned char *gathered, int world, int rows_per, int W, int H, int block,
                            unsigned char *image, void *hip_stream);

/* The P3 writer's pixel values (main.cpp:760, rth_quantize) of n floats as
 * bytes, on the device: out[i] = (int)(rgb[i] * 255) when that is 0..255;
 * otherwise (NaN, values above 1 or below 0 -- the writer prints those as
 * other integers) out[i] = 0 and bit 0 of *flag is set, and the caller must
 * keep the floats.  rgb 16-byte, out 4-byte aligned, device memory;
 * asynchronous on hip_stream.  A multi-GPU render gathers these 3 bytes per
 * pixel instead of 12 (rtamd/dist.py ImageGather, bench.py). */
int rt_quantize_u8(const float *rgb, long long n, unsigned char *out, unsigned *flag, void *hip_stream);

/* Kernel selection / tuning knobs: "accel" (-1 auto, 0 brute-force scan,
 * 1 BVH), "lds" (-1 auto, 0/1: stage the scan's scene in LDS), "grid"
 * (persistent blocks, 0 = occupancy), "reserve" (block slots the occupancy-
 * sized grid leaves free, e.g. for a collective's kernel that must run beside
 * a persistent render), "depth" (recursion depth override),
 * "inflight" (1..8, default 1: renders of this scene that may run at once.
 * With n > 1 each render gets its own work counter, counters and ShadeRay
 * frame buffer and runs on a library stream, ordered against its caller's
 * stream by events: renders issued on different caller streams -- independent
 * frames -- overlap, so one frame's tail is filled by the next frame's work),
 * "frame_share" (-1 auto, 1..8: the occupancy-sized grid is divided by this,
 * so renders in flight run side by side on a share of the CUs each; auto =
 * 2 with inflight > 1 for a render with at most 32 pixels per lane of the
 * occupancy-sized grid -- C3's rows of one rank at N >= 2 --, else 1; ignored when
 * "grid" is set -- never changes the image),
 * "lds_stack" (12..16, default 15: BVH stack entries kept in LDS per lane;
 * deeper stacks spill to device memory -- a test knob), "bvh_leaf" (largest
 * leaf), "bvh_collapse" (0 greedy, 1 SAH-optimal 4-wide collapse), "bvh_node"
 * (the collapse's node cost x1000), "bvh_threads" (host threads of the BVH
 * build: 0 automatic -- the process's CPUs, at most OMP_NUM_THREADS and 16 --,
 * 1 serial; every count builds the same tree),
 * "chunk" (0..4096: pixels a wave takes from the work counter at a time,
 * default 0 = as many as it has idle lanes -- never changes the image),
 * "refill_min" (1..64: idle lanes a wave gathers before it refills them;
 * default 32 when some material reflects or refracts, 48 above depth 4,
 * 64 with primary and shadow rays only), "gate_x"
 * (0..64, default 32: reflection / refraction searches wait until that many
 * lanes of the wave have one, unless nothing else would search) -- neither
 * changes the image,
 * "work_parts" (-1 auto, 1 / 2 / 4 / 8: bands of the work items with a pixel counter
 * each; auto = 8, one per XCD, when the launch has a workgroup per band --
 * never changes the image),
 * "org_first" (-1 auto, or bits 1 shadow / 2 refraction / 4 reflection rays:
 * test the ray's origin object's BVH leaf before the search from the root;
 * auto = 6 in dense scenes, else 0 -- never changes the image),
 * "bvh_presplit" (0..8, default 0: faces whose shadow factor is 0 or 1 enter
 * the BVH as up to that many references with clipped boxes -- never changes
 * the image; measured per scene, not a default),
 * "counters" (1, the default: the kernel instantiation that counts rays and
 * executed tests for rt_stats; 0: the one without counters, which bench.py
 * times -- its stats report no rays; never changes the image),
 * "last_light_skip" (-1 auto, 0 off: a last light whose Phong term is exactly
 * 0 is counted but not searched, in scenes where that is exact -- never
 * changes the image), "recursive" (test hook: 1 renders a scene without
 * reflecting / refracting materials with the recursive instantiation instead
 * of the MAXF = 1 one -- never changes the image),
 * "fail_bvh_upload" (test hook: 1 makes BVH uploads fail with RT_E_NOMEM). */
int rt_scene_set_option(rt_scene *scene, const char *key, long long value);

/* Raw counters of the last render (diagnostics): [0..8] as in rt_stats,
 * [9..15] per-wave cycle / occupancy counters of an RT_PROF build (zero
 * otherwise), then launch facts: [16] kernel mode (0 scan, 1 LDS scan, 2 BVH),
 * [17] resident blocks per CU, [18] grid, [19] LDS bytes per block,
 * [20] BVH nodes, [21] BVH depth, [22] BVH worst-case stack, [23] CUs;
 * launch timeline (100 MHz ticks): [24] first wave start, [26] last wave end;
 * RT_PROF builds also [25] work counter drained, [27] sum of per-wave tails, [28] sum of wave
 * lifetimes, [29] waves; [32] known-zero shadow rays, [33] brute-force queries, [34] stack
 * spills (as in rt_stats), [35] BVH queries with a NaN origin or direction
 * (no hit; not searched; counting instantiation only); RT_PROF builds: [36..38] traversal trips of primary /
 * shadow / refraction + reflection queries, [39] trace steps whose wave searched
 * primary and other rays together; more launch facts: [40] origin-leaf pass
 * bits in effect (option org_first), [41] the scene's density (objects a line
 * across it meets, x1000), [42] BVH stack entries in LDS, [43] lights staged
 * in LDS (1) or read from device memory (0), [44] 0 (on the device this slot
 * counts the ub_back events, which rt_scene_debug_ub_pixels returns; rounds
 * 4-5 reported the removed option hot_copies here), [45] work bands (option
 * work_parts), [46] frames per lane of the kernel instantiation (1, 5, 9 or
 * 17: by depth; 17 also for depth <= 8 with more than 32767 lights), [47] its
 * frame slots split (1: 16-B colour slots apart from the stack slots) or not, [48] the counting kernel instantiation (option counters: 1)
 * or the one without counters (0); RT_CHECK builds: [49] stack-bottom
 * invariant violations (must be 0).  n <= 64. */
int rt_scene_debug_counters(rt_scene *scene, unsigned long long *out, int n);

/* The last render's back() reads of an empty medium stack (main.cpp:1028,
 * undefined behaviour in the reference; defined here as eta_bkg): writes the
 * (x, y) image coordinates of the first min(events, n, 4096) events' pixels
 * into xy[2k], xy[2k+1] (a pixel repeats once per event) and returns the
 * number of events (rt_stats.ub_back), or a negative RT_E_* code. */
int rt_scene_debug_ub_pixels(rt_scene *scene, int *xy, int n);

/* Debug: the last render's per-wave timeline, RT_PROF builds only (others
 * return RT_E_INVALID).  8 words per wave of the launch: [0] wave start,
 * [1] prologue done, [2] work counter seen drained (0: never), [3] wave end
 * (100 MHz ticks, the clock of counters [24..29]), [4] end of the wave's first
 * trace step, [5] HW_ID << 32 | XCC_ID, [6] outer iterations (trace steps),
 * [7] refill batches.  Copies at most n
 * words; returns the number copied. */
int rt_scene_debug_wavelog(rt_scene *scene, unsigned long long *out, int n);

const char *rt_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
