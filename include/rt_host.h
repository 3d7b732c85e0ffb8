/*
 * rt_host.h -- C ABI of the host-side front end that surrounds the GPU layer:
 * the scene-file parser, the camera, quantisation and the P3 PPM writer.
 *
 * These replace, with the same behaviour, the reference's
 *   - scene parser          main.cpp:88-602 (keywords src/config.h:17-50)
 *   - P3 texture reader     src/utility.h:59-139 (read_texture)
 *   - camera                main.cpp:677-710 (inside create_view_window_and_ray_trace)
 *   - quantisation          main.cpp:760-762 (static_cast<int>(map(c,0,1,0,255)))
 *   - PPM writer            main.cpp:613-650 (+ remove_extension, src/utility.h:34-41)
 * Pure C++ (no HIP); librt_host.so.
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rth_scene rth_scene;

/* Parse a scene file.  Texture paths are relative to the current working
 * directory, like the reference.  Returns
 *    0  success (*out set)
 *   >0  the reference would print `msg` on stdout and exit 0 without an image
 *       (unreadable input file, missing required command: main.cpp:567, :574-602)
 *   <0  the reference would throw (std::terminate): `msg` holds the
 *       std::cerr lines it prints, newline separated. */
int rth_parse_file(const char *path, rth_scene **out, char *msg, int msglen);
void rth_free(rth_scene *s);

/* The description to hand to rt_scene_create (valid while `s` lives). */
const rt_scene_desc *rth_desc(const rth_scene *s);
/* Mutable knobs (new CLI flags; the reference hard-codes depth 4). */
void rth_set_depth(rth_scene *s, int depth);
void rth_set_imsize(rth_scene *s, int width, int height);
/* imsize width/height as parsed (or overridden). */
int rth_width(const rth_scene *s);
int rth_height(const rth_scene *s);

/* main.cpp:677-710 for this scene's eye/viewdir/updir/hfov at W x H. */
int rth_camera(const rth_scene *s, int W, int H, rt_camera *cam);

/* main.cpp:760-762 on x86-64: (int)(c * 255) with NaN/out-of-range -> INT_MIN,
 * widened like the reference's size_t element (as int64 here). */
void rth_quantize(const float *rgb, long long n, long long *out);

/* Write the reference's ASCII P3 file for a W x H float image:
 * "P3 \n" "W H \n" "255 \n" then "r g b \n" per pixel, each value the
 * size_t of rth_quantize.  threads <= 0: all cores.  Returns 0 or -1. */
int rth_write_ppm(const char *path, const float *rgb, int W, int H, int threads);

/* The same file written in row blocks, in order (the CLI overlaps each
 * block's device->host copy with the previous block's formatting):
 * rth_ppm_open writes the header; rth_ppm_write_rows appends the next nrows
 * rows (nrows * W * 3 floats); rth_ppm_close returns 0 only when all H rows
 * were written without error.  Byte-identical to rth_write_ppm.  Each returns
 * 0 or -1. */
typedef struct rth_ppm_stream rth_ppm_stream;
int rth_ppm_open(const char *path, int W, int H, int threads, rth_ppm_stream **out);
int rth_ppm_write_rows(rth_ppm_stream *stream, const float *rgb, int nrows);
int rth_ppm_close(rth_ppm_stream *stream);

/* The same file from the pixel values as bytes (W * H * 3, or nrows * W * 3
 * for a row block) -- what rt_hip.h's rt_quantize_u8 makes on the device when
 * every value is 0..255 (its flag clear): byte-identical to rth_write_ppm /
 * rth_ppm_write_rows of the floats they came from.  The CLI copies these
 * 3 bytes per pixel to the host instead of 12.  Each returns 0 or -1. */
int rth_write_ppm_u8(const char *path, const unsigned char *v, int W, int H, int threads);
int rth_ppm_write_rows_u8(rth_ppm_stream *stream, const unsigned char *v, int nrows);

/* remove_extension(path) + ".ppm" (src/utility.h:34-41, main.cpp:614-616). */
int rth_output_path(const char *scene_path, char *out, int outlen);

/* Multi-device row sharding of a H-row image (the reference's row loop
 * main.cpp:718, split): rows are dealt in blocks of `block` rows round robin,
 * so device `rank` of `world` renders local rows k = 0..nrows-1 = image rows
 * y0 + (k / block) * step + k % block, with y0 = rank * block and
 * step = block * world (the arguments of rt_render_row_blocks).  rows_per is
 * the largest rank's row count (equal-size buffers for one gather).  Returns
 * 0, or -1 for bad arguments. */
int rth_row_set(int H, int world, int rank, int block, int *y0, int *step, int *nrows, int *rows_per);

#ifdef __cplusplus
}
#endif
#endif /* RT_HOST_H */
