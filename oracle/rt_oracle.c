/*
 * rt_oracle.c -- CPU restatement of zachoines/simple-raytracer's per-pixel
 * ray-trace path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.  The
 * product (simple-raytracer_amd/, the HIP path) never links or calls it.
 *
 * It restates, in plain C with the reference's float/double conversions:
 *   - the scene-file parser            main.cpp:88-602, src/config.h:17-50
 *   - the P3 texture reader            src/utility.h:59-139
 *   - the camera / pixel loop          main.cpp:670-767
 *   - TraceRay (intersection)          main.cpp:1215-1407
 *   - ShadeRay (shade + recursion)     main.cpp:783-1207
 *   - the PPM writer + quantisation    main.cpp:613-650, :760-762
 * and adds per-type ray counters (one "ray" = one TraceRay call).
 *
 * Pinning: tests/test_oracle.py checks this oracle byte-for-byte against PPMs
 * produced by the real reference (oracle/_ref/SimpleRayTracer, compiled from
 * /root/reference/main.cpp by oracle/Makefile) stored as fixtures in
 * tests/golden/.
 *
 * Build: must be compiled without FMA contraction (-ffp-contract=off) on
 * x86-64, like the reference (SSE scalar float, no FMA).
 */
#include <errno.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_PI 3.14159265358979323846 /* src/config.h:11 */
#define OR_D 5.0                     /* src/config.h:8 view-plane distance */

/* ------------------------------------------------------------------ */
/* Vector3 / Color semantics  (src/definitions.h:18-195)               */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { float r, g, b; } col;

static v3 vadd(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static v3 vsub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static v3 vmulf(v3 a, float f) { v3 r = {a.x * f, a.y * f, a.z * f}; return r; }
static v3 vmulv(v3 a, v3 b) { v3 r = {a.x * b.x, a.y * b.y, a.z * b.z}; return r; }
static v3 vdivf(v3 a, float f) { v3 r = {a.x / f, a.y / f, a.z / f}; return r; }
static float vsum(v3 a) { return a.x + a.y + a.z; }             /* definitions.h:24 */
static float vdot(v3 a, v3 b) { return vsum(vmulv(a, b)); }      /* :29 */
static float vmag(v3 a) { return sqrtf(vsum(vmulv(a, a))); }     /* :34 */
static v3 vnorm(v3 a) { return vdivf(a, vmag(a)); }              /* :57 */
static v3 vcross(v3 a, v3 b) {                                   /* :48 */
    v3 r;
    r.x = a.y * b.z - a.z * b.y;
    r.y = a.z * b.x - a.x * b.z;
    r.z = a.x * b.y - a.y * b.x;
    return r;
}
/* std::clamp(v, 0, 1): (v < lo) ? lo : (hi < v) ? hi : v -- NaN passes through */
static float clamp01(float v) { return (v < 0.0f) ? 0.0f : (1.0f < v) ? 1.0f : v; }
static float clampf(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }
static col cmulc(col a, col b) { col r = {clamp01(b.r * a.r), clamp01(b.g * a.g), clamp01(b.b * a.b)}; return r; }
static col cmulf(col a, float f) { col r = {clamp01(f * a.r), clamp01(f * a.g), clamp01(f * a.b)}; return r; }
static col cadd(col a, col b) { col r = {clamp01(b.r + a.r), clamp01(b.g + a.g), clamp01(b.b + a.b)}; return r; }
static float fmax0(float x) { return (0.0f < x) ? x : 0.0f; }   /* std::max(0.0f, x) */
/* utility.h:23 map() -- all float */
static float mapf(float x, float in_min, float in_max, float out_min, float out_max) {
    return (x - in_min) * (out_max - out_min) / (in_max - in_min) + out_min;
}

/* ------------------------------------------------------------------ */
/* Scene                                                                */
/* ------------------------------------------------------------------ */
typedef struct {
    col diffuse, specular;
    float ka, kd, ks, n, opacity, eta;
} material;

typedef struct {
    int width, height;
    unsigned char *rgb; /* [y][x][3] */
    int *wide;          /* non-NULL when a texel value does not fit a byte */
} texture;

typedef struct {
    int is_sphere;
    material mat;
    int tex;            /* -1: no texture */
    /* sphere */
    v3 center; float radius;
    /* face */
    v3 vert[3], vn[3];
    float vt[3][2];
    int smooth;
    v3 surface_normal;
} object;

typedef struct {
    v3 position, direction; float w; col color;
} light;

typedef struct or_scene {
    int n_obj;          /* faces first (file order), then spheres (file order): main.cpp:1218 */
    object *obj;
    int n_faces, n_spheres;
    int n_lights;
    light *lights;
    int n_tex;
    texture *tex;
    v3 eye, viewdir, updir;
    float fov;
    int width, height;
    col bkg;
    float eta_bkg;      /* environment.other["bkg_refraction_index"], 0 unless given (main.cpp:751) */
    float epsilon;      /* main.cpp:101 */
    int depth;          /* main.cpp:100 */
} or_scene;

/* ------------------------------------------------------------------ */
/* growable arrays                                                      */
/* ------------------------------------------------------------------ */
typedef struct { void *p; int n, cap; size_t esz; } vec_t;
static void *vec_push(vec_t *v) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 64;
        v->p = realloc(v->p, (size_t)v->cap * v->esz);
    }
    void *e = (char *)v->p + (size_t)v->n * v->esz;
    memset(e, 0, v->esz);
    v->n++;
    return e;
}

/* ------------------------------------------------------------------ */
/* std::stof / std::stoi semantics                                      */
/* ------------------------------------------------------------------ */
static int p_stof(const char *s, float *out) {
    char *end;
    errno = 0;
    float f = strtof(s, &end);
    if (end == s) return -1;
    if (errno == ERANGE) return -1;
    *out = f;
    return 0;
}
static int p_stoi(const char *s, int *out) {
    char *end;
    errno = 0;
    long l = strtol(s, &end, 10);
    if (end == s) return -1;
    if (errno == ERANGE || l < INT_MIN || l > INT_MAX) return -1;
    *out = (int)l;
    return 0;
}

/* ------------------------------------------------------------------ */
/* P3 texture reader  (src/utility.h:59-139)                            */
/* ------------------------------------------------------------------ */
static int read_texture(const char *path, texture *t, char *err, int errlen) {
    FILE *f = fopen(path, "rb");
    if (!f) { snprintf(err, errlen, "cannot open texture '%s'", path); return -1; }
    size_t cap = 1 << 20, len = 0;
    char *buf = malloc(cap);
    size_t r;
    while ((r = fread(buf + len, 1, cap - len, f)) > 0) {
        len += r;
        if (len == cap) { cap *= 2; buf = realloc(buf, cap); }
    }
    fclose(f);
    buf[len] = 0;
    int ntok = 0, w = 0, h = 0;
    size_t nval = 0, vcap = 1 << 16;
    long *vals = malloc(vcap * sizeof(long));
    char *line = buf;
    int rc = 0;
    while (line < buf + len) {
        char *nl = memchr(line, '\n', (size_t)(buf + len - line));
        char *lend = nl ? nl : buf + len;
        if (lend == line) { /* line.at(0) on an empty line throws */
            snprintf(err, errlen, "empty line in texture '%s'", path); rc = -1; break;
        }
        if (line[0] != '#') {
            char *p = line;
            while (p <= lend) {
                char *sp = p;
                while (sp < lend && *sp != ' ') sp++;
                if (sp > p) {
                    char save = *sp; *sp = 0;
                    ntok++;
                    if (ntok == 1) {
                        if (strcmp(p, "P3") != 0) { snprintf(err, errlen, "Only supports PPM 'P3' file format."); rc = -1; }
                    } else if (ntok == 2) {
                        if (p_stoi(p, &w)) rc = -1;
                    } else if (ntok == 3) {
                        if (p_stoi(p, &h)) rc = -1;
                    } else if (ntok == 4) {
                        if (strcmp(p, "255") != 0) { snprintf(err, errlen, "PPM pixel value must be between 0 - 255 ."); rc = -1; }
                    } else {
                        int iv = 0;
                        if (p_stoi(p, &iv)) { rc = -1; }
                        if (nval == vcap) { vcap *= 2; vals = realloc(vals, vcap * sizeof(long)); }
                        vals[nval++] = iv;
                    }
                    *sp = save;
                    if (rc) break;
                }
                p = sp + 1;
            }
        }
        if (rc) break;
        line = lend + 1;
    }
    free(buf);
    if (!rc && (w <= 0 || h <= 0 || nval < (size_t)w * h * 3)) {
        snprintf(err, errlen, "texture '%s' truncated", path); rc = -1;
    }
    if (rc) { free(vals); return -1; }
    t->width = w; t->height = h;
    t->rgb = malloc((size_t)w * h * 3);
    t->wide = NULL;
    for (size_t i = 0; i < (size_t)w * h * 3; i++) {
        if (vals[i] < 0 || vals[i] > 255) {
            if (!t->wide) {
                t->wide = malloc((size_t)w * h * 3 * sizeof(int));
                for (size_t k = 0; k < i; k++) t->wide[k] = t->rgb[k];
            }
        }
        t->rgb[i] = (unsigned char)vals[i];
        if (t->wide) t->wide[i] = (int)vals[i];
    }
    free(vals);
    return 0;
}

/* texel (x, y, c) -> float, main.cpp:823/858: map(size_t, 0, 255, 0, 1) */
static float texel(const texture *t, int x, int y, int c) {
    size_t i = ((size_t)y * t->width + x) * 3 + c;
    float v = t->wide ? (float)(size_t)(long)t->wide[i] : (float)t->rgb[i];
    return mapf(v, 0.0f, 255.0f, 0.0f, 1.0f);
}

/* ------------------------------------------------------------------ */
/* Scene parser  (main.cpp:88-602)                                      */
/* ------------------------------------------------------------------ */
enum { K_EYE, K_VIEWDIR, K_UPDIR, K_HFOV, K_IMSIZE, K_BKG, K_MTL, K_TEX, K_SPHERE, K_LIGHT, K_V, K_VN, K_VT, K_F, K_NONE };
static int keyword(const char *s) {
    static const char *kw[] = {"eye", "viewdir", "updir", "hfov", "imsize", "bkgcolor", "mtlcolor",
                               "texture", "sphere", "light", "v", "vn", "vt", "f"};
    for (int i = 0; i < 14; i++) if (strcmp(s, kw[i]) == 0) return i;
    return K_NONE;
}

#define MAXTOK 64
static int parse_floats(char **a, int na, int from, int cnt, float *out) {
    for (int i = 0; i < cnt; i++) {
        if (from + i >= na) return -1;
        if (p_stof(a[from + i], &out[i])) return -1;
    }
    return 0;
}

void oracle_free(or_scene *s);

/* Returns 0 on success.  Negative on an error that aborts the reference
 * (exception -> std::terminate); positive 1 on a "missing command" message
 * (reference prints and exits 0 without writing an image). */
int oracle_load(const char *path, or_scene **out, char *err, int errlen) {
    *out = NULL;
    FILE *f = fopen(path, "rb");
    if (!f) { snprintf(err, errlen, "ERROR: Issue reading input file '%s'. Please verify path.", path); return 2; }
    or_scene *S = calloc(1, sizeof(or_scene));
    S->epsilon = 1.0e-3f; S->depth = 4; S->eta_bkg = 0.0f;
    vec_t verts = {0, 0, 0, sizeof(v3)}, norms = {0, 0, 0, sizeof(v3)}, tcs = {0, 0, 0, 2 * sizeof(float)};
    vec_t faces = {0, 0, 0, sizeof(object)}, sphs = {0, 0, 0, sizeof(object)};
    vec_t lights = {0, 0, 0, sizeof(light)}, texs = {0, 0, 0, sizeof(texture)};
    int seen[6] = {0};
    material cur_mat; memset(&cur_mat, 0, sizeof cur_mat);
    int has_mat = 0, use_tex = 0, cur_tex = -1;
    char line[1 << 16];
    int rc = 0;
    while (fgets(line, sizeof line, f)) {
        size_t L = strlen(line);
        if (L && line[L - 1] == '\n') line[--L] = 0;
        if (L == 0) continue;
        /* split on single ' '; an empty token throws from del.at(0) (main.cpp:114) */
        char *tok[MAXTOK]; int nt = 0;
        char *p = line;
        for (;;) {
            char *sp = strchr(p, ' ');
            if (!sp) {
                if (*p == 0) break;     /* trailing delimiter: getline stops */
                if (nt < MAXTOK) tok[nt++] = p;
                break;
            }
            *sp = 0;
            if (*p == 0) { snprintf(err, errlen, "basic_string::at: empty token"); rc = -1; goto done; }
            if (nt < MAXTOK) tok[nt++] = p;
            p = sp + 1;
        }
        if (nt == 0) continue;
        int k = keyword(tok[0]);
        char **a = tok + 1; int na = nt - 1;
        if (na == 0 || k == K_NONE) continue;
        float fv[12];
        switch (k) {
        case K_EYE: case K_VIEWDIR: case K_UPDIR:
            seen[k] = 1;
            if (parse_floats(a, na, 0, 3, fv)) { rc = -1; goto bad; }
            {
                v3 v = {fv[0], fv[1], fv[2]};
                if (k == K_EYE) S->eye = v; else if (k == K_VIEWDIR) S->viewdir = v; else S->updir = v;
            }
            break;
        case K_HFOV:
            seen[K_HFOV] = 1;
            if (parse_floats(a, na, 0, 1, fv)) { rc = -1; goto bad; }
            S->fov = fv[0];
            break;
        case K_IMSIZE: {
            seen[K_IMSIZE] = 1;
            int w, h;
            if (na < 2 || p_stoi(a[1], &h) || p_stoi(a[0], &w)) { rc = -1; goto bad; }
            if (h <= 1 || w <= 1) { rc = -1; goto bad; }
            S->width = w; S->height = h;
            break;
        }
        case K_BKG:
            seen[K_BKG] = 1;
            if (parse_floats(a, na, 0, 3, fv)) { rc = -1; goto bad; }
            S->bkg.r = fv[0]; S->bkg.g = fv[1]; S->bkg.b = fv[2];
            if (na > 3) {
                if (p_stof(a[3], &fv[3])) { rc = -1; goto bad; }
                S->eta_bkg = fv[3];
            }
            break;
        case K_MTL: {
            use_tex = 0;
            material m;
            if (parse_floats(a, na, 0, 10, fv)) { rc = -1; goto bad; }
            m.diffuse.r = fv[0]; m.diffuse.g = fv[1]; m.diffuse.b = fv[2];
            m.specular.r = fv[3]; m.specular.g = fv[4]; m.specular.b = fv[5];
            m.ka = fv[6]; m.kd = fv[7]; m.ks = fv[8]; m.n = fv[9];
            if (na == 12) {
                if (parse_floats(a, na, 10, 2, fv + 10)) { rc = -1; goto bad; }
                m.opacity = clampf(fv[10], 0.0f, 1.0f);
                m.eta = fv[11];
            } else {
                m.opacity = 1.0f; m.eta = 1.0f;
            }
            cur_mat = m; has_mat = 1;
            break;
        }
        case K_TEX: {
            use_tex = 1;
            texture *t = vec_push(&texs);
            if (read_texture(a[0], t, err, errlen)) { texs.n--; rc = -1; goto done; }
            cur_tex = texs.n - 1;
            break;
        }
        case K_SPHERE: {
            if (parse_floats(a, na, 0, 4, fv)) { rc = -1; goto bad; }
            object *o = vec_push(&sphs);
            o->is_sphere = 1;
            o->radius = fv[3];
            o->center.x = fv[0]; o->center.y = fv[1]; o->center.z = fv[2];
            o->mat = cur_mat;
            o->tex = -1;
            if (use_tex) {
                if (!has_mat || cur_tex < 0) { rc = -1; goto bad; }
                o->tex = cur_tex;
            } else if (!has_mat) { rc = -1; goto bad; }
            break;
        }
        case K_LIGHT: {
            if (parse_floats(a, na, 0, 7, fv)) { rc = -1; goto bad; }
            light *l = vec_push(&lights);
            l->w = fv[3];
            v3 v = {fv[0], fv[1], fv[2]};
            if (l->w == 0) l->direction = v; else l->position = v;
            l->color.r = fv[4]; l->color.g = fv[5]; l->color.b = fv[6];
            break;
        }
        case K_V: case K_VN: {
            if (parse_floats(a, na, 0, 3, fv)) { rc = -1; goto bad; }
            v3 *v = vec_push(k == K_V ? &verts : &norms);
            v->x = fv[0]; v->y = fv[1]; v->z = fv[2];
            break;
        }
        case K_VT: {
            if (parse_floats(a, na, 0, 2, fv)) { rc = -1; goto bad; }
            float *t = vec_push(&tcs);
            t[0] = fv[0]; t[1] = fv[1];
            break;
        }
        case K_F: {
            object *o = vec_push(&faces);
            o->is_sphere = 0;
            o->tex = -1;
            if (na < 3) { rc = -1; goto bad; }
            for (int i = 0; i < 3; i++) {
                unsigned int v, t, n;
                const v3 *V = verts.p, *N = norms.p;
                const float (*T)[2] = tcs.p;
                v3 zero = {0, 0, 0};
#define VERT(ix) (((ix) >= 1 && (int)(ix) <= verts.n) ? V[(ix) - 1] : zero)
#define NORM(ix) (((ix) >= 1 && (int)(ix) <= norms.n) ? N[(ix) - 1] : zero)
                if (sscanf(a[i], "%d/%d/%d", (int *)&v, (int *)&t, (int *)&n) == 3) {
                    o->vert[i] = VERT(v); o->vn[i] = NORM(n); o->smooth = 1;
                    if (t >= 1 && (int)t <= tcs.n) { o->vt[i][0] = T[t - 1][0]; o->vt[i][1] = T[t - 1][1]; }
                    else { o->vt[i][0] = 0; o->vt[i][1] = 0; }
                } else if (sscanf(a[i], "%d//%d", (int *)&v, (int *)&n) == 2) {
                    o->vert[i] = VERT(v); o->vn[i] = NORM(n); o->smooth = 1;
                } else if (sscanf(a[i], "%d/%d", (int *)&v, (int *)&t) == 2) {
                    o->vert[i] = VERT(v); o->smooth = 0;
                    if (t >= 1 && (int)t <= tcs.n) { o->vt[i][0] = T[t - 1][0]; o->vt[i][1] = T[t - 1][1]; }
                    else { o->vt[i][0] = 0; o->vt[i][1] = 0; }
                } else if (sscanf(a[i], "%d", (int *)&v) == 1) {
                    o->vert[i] = VERT(v); o->smooth = 0;
                } else { rc = -1; goto bad; }
#undef VERT
#undef NORM
            }
            o->mat = cur_mat;
            if (use_tex) {
                if (!has_mat || cur_tex < 0) { rc = -1; goto bad; }
                o->tex = cur_tex;
            } else if (!has_mat) { rc = -1; goto bad; }
            {
                v3 e1 = vsub(o->vert[1], o->vert[0]);
                v3 e2 = vsub(o->vert[2], o->vert[0]);
                o->surface_normal = vnorm(vcross(e1, e2));  /* main.cpp:537-539 */
            }
            break;
        }
        }
        continue;
    bad:
        snprintf(err, errlen, "ERROR: Command '%s' is undefined. Please verify input.", tok[0]);
        goto done;
    }
done:
    fclose(f);
    if (rc == 0) {
        static const char *names[] = {"imsize", "eye", "viewdir", "updir", "hfov", "bkgcolor"};
        static const int keys[] = {K_IMSIZE, K_EYE, K_VIEWDIR, K_UPDIR, K_HFOV, K_BKG};
        for (int i = 0; i < 6; i++)
            if (!seen[keys[i]]) { snprintf(err, errlen, "Error: Requires command '%s'", names[i]); rc = 1; break; }
    }
    S->n_faces = faces.n; S->n_spheres = sphs.n;
    S->n_obj = faces.n + sphs.n;
    S->obj = malloc(sizeof(object) * (size_t)(S->n_obj ? S->n_obj : 1));
    if (faces.n) memcpy(S->obj, faces.p, sizeof(object) * (size_t)faces.n);
    if (sphs.n) memcpy(S->obj + faces.n, sphs.p, sizeof(object) * (size_t)sphs.n);
    S->n_lights = lights.n; S->lights = lights.p;
    S->n_tex = texs.n; S->tex = texs.p;
    free(verts.p); free(norms.p); free(tcs.p); free(faces.p); free(sphs.p);
    if (rc != 0) { oracle_free(S); return rc; }
    *out = S;
    return 0;
}

void oracle_free(or_scene *s) {
    if (!s) return;
    for (int i = 0; i < s->n_tex; i++) { free(s->tex[i].rgb); free(s->tex[i].wide); }
    free(s->tex); free(s->obj); free(s->lights); free(s);
}

/* ------------------------------------------------------------------ */
/* TraceRay  (main.cpp:1215-1407)                                       */
/* Intersections are visited in the reference's order: every face in    */
/* file order, then every sphere in file order; a sphere yields the     */
/* (-B + sqrt) root, then the (-B - sqrt) root.                          */
/* ------------------------------------------------------------------ */
typedef struct {
    int obj;          /* object index (order key) */
    float t;
    v3 point, normal;
    v3 bary;          /* faces: (a, b, g) of this ray -- main.cpp:1372 */
} hitrec;

/* face test: returns 1 and fills t/point/normal/bary if the ray hits the
 * triangle's interior (edges miss). */
static int face_test(const object *F, v3 o, v3 d, hitrec *h) {
    v3 e1 = vsub(F->vert[1], F->vert[0]);
    v3 e2 = vsub(F->vert[2], F->vert[0]);
    v3 n = F->surface_normal;
    float dem = vdot(n, d);
    if (dem == 0.0f) return 0;
    float D = -vdot(n, F->vert[0]);
    float t = -(vdot(n, o) + D) / dem;
    v3 p = vadd(o, vmulf(d, t));
    v3 ep = vsub(p, F->vert[0]);
    float d11 = vdot(e1, e1), d12 = vdot(e1, e2), d22 = vdot(e2, e2);
    float d1p = vdot(e1, ep), d2p = vdot(e2, ep);
    float det = (d11 * d22 - d12 * d12);
    if (det == 0.0f) return 0;
    float b = (d22 * d1p - d12 * d2p) / det;
    float g = (d11 * d2p - d12 * d1p) / det;
    float a = 1.0f - (b + g);
    if (!(((0.0f < a) && (a < 1.0f)) && ((0.0f < b) && (b < 1.0f)) && ((0.0f < g) && (g < 1.0f)))) return 0;
    v3 nn;
    if (F->smooth) {
        nn = vnorm(vadd(vadd(vmulf(vnorm(F->vn[0]), a), vmulf(vnorm(F->vn[1]), b)), vmulf(vnorm(F->vn[2]), g)));
    } else {
        nn = F->surface_normal;
    }
    h->t = t; h->point = p; h->normal = nn;
    h->bary.x = a; h->bary.y = b; h->bary.z = g;
    return 1;
}

/* sphere test: returns the number of roots pushed (0 or 2), in order */
static int sphere_test(const object *S, v3 o, v3 d, float t[2]) {
    v3 dir = vsub(o, S->center);
    float B = (float)(2.0 * (double)vsum(vmulv(d, dir)));
    float C = (float)((double)vsum(vmulv(dir, dir)) - (double)S->radius * (double)S->radius);
    float det = (float)((double)B * (double)B - (4.0 * 1.0 * (double)C));
    if (!signbit(det)) {
        t[0] = (float)((double)(-B + sqrtf(det)) / 2.0);
        t[1] = (float)((double)(-B - sqrtf(det)) / 2.0);
        return 2;
    }
    return 0;
}

static void sphere_hit(const object *S, v3 o, v3 d, float t, hitrec *h) {
    h->t = t;
    h->point = vadd(o, vmulf(d, t));
    h->normal = vnorm(vdivf(vsub(h->point, S->center), S->radius));
}

typedef struct {
    long long prim, shadow, refr, refl;  /* TraceRay calls by type */
    long long skip;                      /* SKIP_TRANS taken (main.cpp:1001) */
    long long ub_back;                   /* back() on empty stack (main.cpp:1028) */
} counters;

/* closest intersection with tmin < t < running min, visiting in order.
 * When skip_back >= 0 the SKIP_TRANS rule (main.cpp:1000-1002) applies: a
 * record-breaking intersection on an object other than skip_back aborts.
 * Returns 1 hit, 0 miss, 2 skip. */
static int closest(const or_scene *S, v3 o, v3 d, float tmin, int skip_back, hitrec *best) {
    float min_d = 3.40282347e+38f;
    int found = 0;
    for (int i = 0; i < S->n_obj; i++) {
        const object *ob = &S->obj[i];
        if (!ob->is_sphere) {
            hitrec h;
            if (face_test(ob, o, d, &h)) {
                if (h.t > tmin && h.t < min_d) {
                    if (skip_back >= 0 && i != skip_back) return 2;
                    min_d = h.t; *best = h; best->obj = i; found = 1;
                }
            }
        } else {
            float t[2];
            int n = sphere_test(ob, o, d, t);
            for (int k = 0; k < n; k++) {
                if (t[k] > tmin && t[k] < min_d) {
                    if (skip_back >= 0 && i != skip_back) return 2;
                    min_d = t[k];
                    sphere_hit(ob, o, d, t[k], best);
                    best->obj = i; found = 1;
                }
            }
        }
    }
    if (found) {
        /* recompute bary of the winning face exactly as its trace did */
        return 1;
    }
    return 0;
}

/* shadow scan: every intersection of every object except self with
 * tmin < t (and t < tmax when bounded) multiplies the mask by (1 - opacity),
 * main.cpp:896-912 and :928-949 */
static col shadow(const or_scene *S, v3 o, v3 d, int self, float eps, int bounded, float tmax, col mask) {
    for (int i = 0; i < S->n_obj; i++) {
        const object *ob = &S->obj[i];
        float t[2]; int n;
        if (!ob->is_sphere) {
            hitrec h;
            n = face_test(ob, o, d, &h);
            t[0] = h.t;
        } else {
            n = sphere_test(ob, o, d, t);
        }
        if (i == self) continue;
        for (int k = 0; k < n; k++) {
            if (t[k] > eps && (!bounded || t[k] < tmax))
                mask = cmulf(mask, (float)(1.0 - (double)ob->mat.opacity));
        }
    }
    return mask;
}

/* ------------------------------------------------------------------ */
/* ShadeRay  (main.cpp:783-1207)                                        */
/* ------------------------------------------------------------------ */
enum { ENTERING = 0, EXITING = 1 };
#define MAXSTACK 64

static col shade(const or_scene *S, counters *C, v3 ray, int self, const hitrec *hit, float eta_i, float eta_t,
                 const int *stack, int sn, int state, float depth) {
    const object *ob = &S->obj[self];
    material m = ob->mat;
    v3 N = hit->normal;
    v3 I = vmulf(ray, -1.0f);
    col spec = {0, 0, 0}, mask = {1, 1, 1}, diffuse, trans = {0, 0, 0}, refl = {0, 0, 0};
    float cosI = vdot(N, I);
    int prev = state;
    col bkg = S->bkg;

    if (ob->tex >= 0) {                                           /* :800-862 */
        const texture *tx = &S->tex[ob->tex];
        if (ob->is_sphere) {
            float v = (float)(acos((double)N.z) / OR_PI);
            float phi = (float)atan2((double)N.y, (double)N.x);
            float u = mapf(phi, (float)-OR_PI, (float)OR_PI, 0.0f, 1.0f);
            float width = (float)tx->width, height = (float)tx->height;
            v = clampf(v, 0.0f, 1.0f);
            u = clampf(u, 0.0f, 1.0f);
            int i = (int)clampf((float)round(((double)height - 1.0) * (double)v), 0.0f, (float)((double)height - 1.0));
            int j = (int)clampf((float)round(((double)width - 1.0) * (double)u), 0.0f, (float)((double)width - 1.0));
            diffuse.r = texel(tx, j, i, 0); diffuse.g = texel(tx, j, i, 1); diffuse.b = texel(tx, j, i, 2);
        } else {
            v3 bc = hit->bary;
            float u = (bc.x * clampf(ob->vt[0][0], 0.0f, 1.0f)) + (bc.y * clampf(ob->vt[1][0], 0.0f, 1.0f)) +
                      (bc.z * clampf(ob->vt[2][0], 0.0f, 1.0f));
            float v = (bc.x * clampf(ob->vt[0][1], 0.0f, 1.0f)) + (bc.y * clampf(ob->vt[1][1], 0.0f, 1.0f)) +
                      (bc.z * clampf(ob->vt[2][1], 0.0f, 1.0f));
            v = clampf(v, 0.0f, 1.0f);
            u = clampf(u, 0.0f, 1.0f);
            float width = (float)tx->width, height = (float)tx->height;
            int i = (int)clampf(roundf((width - 1.0f) * u), 0.0f, (float)((double)width - 1.0));
            int j = (int)clampf(roundf((height - 1.0f) * v), 0.0f, (float)((double)height - 1.0));
            diffuse.r = texel(tx, i, j, 0); diffuse.g = texel(tx, i, j, 1); diffuse.b = texel(tx, i, j, 2);
        }
    } else {
        diffuse = m.diffuse;
    }

    if ((double)cosI < 0.0 && ob->is_sphere) {                     /* :869-872 */
        N = vmulf(N, -1.0f);
        cosI = vdot(N, I);
    }

    for (int li = 0; li < S->n_lights; li++) {                     /* :878-959 */
        const light *lt = &S->lights[li];
        v3 L, H;
        C->shadow++;
        if (lt->w == 0) {
            L = vmulf(vnorm(lt->direction), -1.0f);
            v3 sray = vmulf(lt->direction, -1.0f);
            mask = shadow(S, hit->point, sray, self, S->epsilon, 0, 0.0f, mask);
        } else {
            L = vnorm(vsub(lt->position, hit->point));
            v3 dl = vsub(hit->point, lt->position);
            float distL = sqrtf(vsum(vmulv(dl, dl)));
            mask = shadow(S, hit->point, L, self, S->epsilon, 1, distL, mask);
        }
        H = vnorm(vadd(L, I));
        col dc = cmulf(cmulf(diffuse, m.kd), fmax0(vdot(N, L)));
        col sc = cmulf(cmulf(m.specular, m.ks), powf(fmax0(vdot(N, H)), m.n));
        spec = cadd(spec, cmulc(cmulc(lt->color, mask), cadd(dc, sc)));
    }

    float snell = eta_i / eta_t;                                   /* :961-966 */
    float crit = asinf(eta_t / eta_i);
    float inc = acosf(cosI);
    int tir = (crit < inc) && ((double)inc < (90.0 * OR_PI / 180.0));
    float F0 = (eta_t - eta_i) / (eta_t + eta_i);
    F0 = F0 * F0;                                                  /* powf(x, 2.0) folds to x*x */
    float F = (float)((double)F0 + (1.0 - (double)F0) * (double)powf((float)(1.0 - (double)cosI), 5.0f));

    if (depth > 0 && !tir && (double)m.opacity < 1.0 && m.eta > 0) {   /* :976-1089 */
        float k = sqrtf((float)(1.0 - (double)(snell * snell) * (1.0 - (double)(cosI * cosI))));
        v3 T = vadd(vmulf(vmulf(N, -1.0f), k), vmulf(vsub(vmulf(N, cosI), I), snell));
        C->refr++;
        int skip_back = (sn > 0 && !ob->is_sphere) ? stack[sn - 1] : -1;
        hitrec h;
        int r = closest(S, hit->point, T, S->epsilon, skip_back, &h);
        if (r == 2) {
            C->skip++;
            goto skip_trans;
        }
        if (r == 1) {
            int ns[MAXSTACK]; int nn = sn;
            memcpy(ns, stack, sizeof(int) * (size_t)sn);
            float ni, nt; int nstate;
            float hit_eta = S->obj[h.obj].mat.eta;
            if (prev == ENTERING) {
                if (h.obj == self) {
                    nstate = EXITING;
                    if (nn > 0) ni = S->obj[ns[nn - 1]].mat.eta;
                    else { ni = S->eta_bkg; C->ub_back++; }   /* back() on empty: UB in the reference */
                    if (nn > 0) nn--;
                    nt = nn > 0 ? S->obj[ns[nn - 1]].mat.eta : S->eta_bkg;
                    if (nn > 0) nn--;
                } else {
                    nstate = ENTERING; ni = eta_t; nt = hit_eta; ns[nn++] = h.obj;
                }
            } else {
                if (nn > 0) {
                    int in = 0;
                    for (int q = 0; q < nn; q++) if (ns[q] == h.obj) in = 1;
                    if (!in) { nstate = ENTERING; ni = eta_t; nt = hit_eta; ns[nn++] = h.obj; }
                    else { nstate = EXITING; ni = eta_t; nt = S->obj[ns[nn - 1]].mat.eta; nn--; }
                } else {
                    nstate = ENTERING; ni = S->eta_bkg; nt = hit_eta; ns[0] = h.obj; nn = 1;
                }
            }
            col c = shade(S, C, T, h.obj, &h, ni, nt, ns, nn, nstate, depth - 1);
            trans = cmulf(cmulf(c, (float)(1.0 - (double)F)), (float)(1.0 - (double)m.opacity));
        } else {
            trans = cmulf(cmulf(bkg, (float)(1.0 - (double)F)), (float)(1.0 - (double)m.opacity));
        }
    }
skip_trans:;

    F0 = (m.eta - 1) / (m.eta + 1);                                /* :1103-1200 */
    F0 = F0 * F0;
    F = (float)((double)F0 + (1.0 - (double)F0) * (double)powf((float)(1.0 - (double)cosI), 5.0f));
    if (depth > 0 && (double)F != 0.0 && (double)m.ks > 0.0) {
        v3 R = vsub(vmulf(N, (float)(2.0 * (double)cosI)), I);
        C->refl++;
        hitrec h;
        if (closest(S, hit->point, R, S->epsilon, -1, &h) == 1) {
            int ns[MAXSTACK]; int nn = sn;
            memcpy(ns, stack, sizeof(int) * (size_t)sn);
            float ni, nt; int nstate;
            float hit_eta = S->obj[h.obj].mat.eta;
            if (prev == ENTERING) {
                if (nn > 0) {
                    int in = 0;
                    for (int q = 0; q < nn; q++) if (ns[q] == h.obj) in = 1;
                    if (!in) { nstate = ENTERING; ni = eta_i; nt = hit_eta; ns[nn++] = self; }
                    else { nstate = ENTERING; ni = eta_i; nt = S->obj[ns[nn - 1]].mat.eta; nn--; }
                } else {
                    nstate = ENTERING; ni = eta_i; nt = hit_eta; ns[0] = h.obj; nn = 1;
                }
            } else {
                if (h.obj == self) { nstate = EXITING; ni = eta_i; nt = eta_t; }
                else { nstate = ENTERING; ni = eta_i; nt = hit_eta; ns[nn++] = h.obj; }
            }
            col c = shade(S, C, R, h.obj, &h, ni, nt, ns, nn, nstate, depth - 1);
            refl = cmulf(c, F);
        } else {
            refl = cmulf(bkg, F);
        }
    }
    return cadd(cadd(cadd(cmulf(diffuse, m.ka), spec), trans), refl);
}

/* ------------------------------------------------------------------ */
/* Camera + pixel loop  (main.cpp:670-767)                              */
/* ------------------------------------------------------------------ */
typedef struct { v3 eye, ul, dh, dv; } camera;

static camera make_camera(const or_scene *S, int W, int H) {
    v3 vd = vnorm(S->viewdir), up = vnorm(S->updir);              /* main.cpp:607 */
    float res_w = (float)W, res_h = (float)H;
    v3 u = vnorm(vcross(vd, up));
    v3 v = vcross(u, vd);
    float aspect = res_w / res_h;
    float w = (float)(2.0f * OR_D * tan((0.5 * (double)S->fov) * OR_PI / 180.0f));
    float h = w / aspect;
    v3 n = vd;
    float df = (float)OR_D;
    v3 ul = vadd(vsub(vadd(S->eye, vmulf(n, df)), vmulf(u, w / 2.0f)), vmulf(v, h / 2.0f));
    v3 ur = vadd(vadd(vadd(S->eye, vmulf(n, df)), vmulf(u, w / 2.0f)), vmulf(v, h / 2.0f));
    v3 ll = vsub(vsub(vadd(S->eye, vmulf(n, df)), vmulf(u, w / 2.0f)), vmulf(v, h / 2.0f));
    camera c;
    c.eye = S->eye;
    c.ul = ul;
    c.dh = vdivf(vsub(ur, ul), res_w - 1.0f);
    c.dv = vdivf(vsub(ll, ul), res_h - 1.0f);
    return c;
}

static col render_pixel(const or_scene *S, const camera *cam, int i, int j, counters *C) {
    v3 p = vadd(vadd(cam->ul, vmulf(cam->dh, (float)j)), vmulf(cam->dv, (float)i));
    col pc = S->bkg;
    v3 ray = vnorm(vsub(p, cam->eye));
    C->prim++;
    hitrec h;
    if (closest(S, cam->eye, ray, 0.0f, -1, &h) == 1) {
        int st[1] = {h.obj};
        pc = shade(S, C, ray, h.obj, &h, S->eta_bkg, S->obj[h.obj].mat.eta, st, 1, ENTERING, (float)S->depth);
    }
    return pc;
}

/* ------------------------------------------------------------------ */
/* public C API (ctypes)                                                */
/* ------------------------------------------------------------------ */
int oracle_width(const or_scene *s) { return s->width; }
int oracle_height(const or_scene *s) { return s->height; }
int oracle_counts_objects(const or_scene *s, int *nf, int *ns, int *nl) {
    *nf = s->n_faces; *ns = s->n_spheres; *nl = s->n_lights; return s->n_obj;
}
void oracle_set_depth(or_scene *s, int depth) { s->depth = depth; }

/* Parsed-scene dump for the host-parser parity test: object i in render
 * order (faces then spheres) as 48 floats:
 *   [0] is_sphere [1] tex [2..13] material (diffuse3 specular3 ka kd ks n opacity eta)
 *   [14..17] center, radius  [18..26] vert[3]  [27..35] vn[3]  [36..41] vt[3]  [42] smooth */
int oracle_object(const or_scene *s, int i, float *o) {
    if (i < 0 || i >= s->n_obj) return -1;
    const object *b = &s->obj[i];
    memset(o, 0, 48 * sizeof(float));
    o[0] = (float)b->is_sphere; o[1] = (float)b->tex;
    const material *m = &b->mat;
    float mm[12] = {m->diffuse.r, m->diffuse.g, m->diffuse.b, m->specular.r, m->specular.g, m->specular.b,
                    m->ka, m->kd, m->ks, m->n, m->opacity, m->eta};
    memcpy(o + 2, mm, sizeof mm);
    o[14] = b->center.x; o[15] = b->center.y; o[16] = b->center.z; o[17] = b->radius;
    for (int k = 0; k < 3; k++) {
        o[18 + 3 * k] = b->vert[k].x; o[19 + 3 * k] = b->vert[k].y; o[20 + 3 * k] = b->vert[k].z;
        o[27 + 3 * k] = b->vn[k].x; o[28 + 3 * k] = b->vn[k].y; o[29 + 3 * k] = b->vn[k].z;
        o[36 + 2 * k] = b->vt[k][0]; o[37 + 2 * k] = b->vt[k][1];
    }
    o[42] = (float)b->smooth;
    return 0;
}

/* lights (8 floats each: xyz w rgb -), bkg/eta_bkg, view */
int oracle_light(const or_scene *s, int i, float *o) {
    if (i < 0 || i >= s->n_lights) return -1;
    const light *l = &s->lights[i];
    v3 p = l->w == 0 ? l->direction : l->position;
    o[0] = p.x; o[1] = p.y; o[2] = p.z; o[3] = l->w; o[4] = l->color.r; o[5] = l->color.g; o[6] = l->color.b;
    o[7] = 0;
    return 0;
}
void oracle_globals(const or_scene *s, float *o) {
    o[0] = s->bkg.r; o[1] = s->bkg.g; o[2] = s->bkg.b; o[3] = s->eta_bkg; o[4] = s->epsilon; o[5] = (float)s->depth;
}
/* camera of main.cpp:677-710 as 12 floats: eye ul dh dv */
void oracle_camera(const or_scene *s, int W, int H, float *o) {
    camera c = make_camera(s, W, H);
    v3 v[4] = {c.eye, c.ul, c.dh, c.dv};
    for (int k = 0; k < 4; k++) { o[3 * k] = v[k].x; o[3 * k + 1] = v[k].y; o[3 * k + 2] = v[k].z; }
}
/* texture i: width, height and a pointer to its [h][w][3] bytes */
int oracle_texture(const or_scene *s, int i, int *w, int *h, const unsigned char **rgb) {
    if (i < 0 || i >= s->n_tex) return -1;
    *w = s->tex[i].width; *h = s->tex[i].height; *rgb = s->tex[i].rgb;
    return 0;
}

/* Render rows rows[0..nrows) of a W x H image into out[nrows][W][3].
 * counts[6] = prim, shadow, refr, refl, skip, ub_back. */
int oracle_render_rows(const or_scene *S, int W, int H, const int *rows, int nrows, int threads, float *out,
                       long long *counts) {
    camera cam = make_camera(S, W, H);
    long long tot[6] = {0};
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads)
#endif
    {
        counters C; memset(&C, 0, sizeof C);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int r = 0; r < nrows; r++) {
            int i = rows[r];
            for (int j = 0; j < W; j++) {
                col c = render_pixel(S, &cam, i, j, &C);
                float *o = out + ((size_t)r * W + j) * 3;
                o[0] = c.r; o[1] = c.g; o[2] = c.b;
            }
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            tot[0] += C.prim; tot[1] += C.shadow; tot[2] += C.refr; tot[3] += C.refl;
            tot[4] += C.skip; tot[5] += C.ub_back;
        }
    }
    for (int k = 0; k < 6; k++) counts[k] = tot[k];
    return 0;
}

/* Render an arbitrary pixel list (x, y pairs) of a W x H image -- the
 * full-size row-span samples of the parity tests (main.cpp:718-764 per pixel). */
int oracle_render_pixels(const or_scene *S, int W, int H, const int *xy, int npx, int threads, float *out,
                         long long *counts) {
    camera cam = make_camera(S, W, H);
    long long tot[6] = {0};
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads)
#endif
    {
        counters C; memset(&C, 0, sizeof C);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int k = 0; k < npx; k++) {
            col c = render_pixel(S, &cam, xy[2 * k + 1], xy[2 * k], &C);
            out[3 * (size_t)k + 0] = c.r; out[3 * (size_t)k + 1] = c.g; out[3 * (size_t)k + 2] = c.b;
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            tot[0] += C.prim; tot[1] += C.shadow; tot[2] += C.refr; tot[3] += C.refl;
            tot[4] += C.skip; tot[5] += C.ub_back;
        }
    }
    for (int k = 0; k < 6; k++) counts[k] = tot[k];
    return 0;
}

/* main.cpp:760: static_cast<int>(map(c, 0, 1, 0, 255)) on x86-64:
 * cvttss2si yields INT_MIN for NaN and out-of-range values. */
static int quantize(float c) {
    float x = mapf(c, 0.0f, 1.0f, 0.0f, 255.0f);
    if (x >= -2147483648.0f && x < 2147483648.0f) return (int)x;
    return INT_MIN;
}

/* Write the reference's P3 format (main.cpp:628-648). */
int oracle_write_ppm(const char *path, const float *rgb, int W, int H) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "P3 \n%d %d \n255 \n", W, H);
    for (size_t i = 0; i < (size_t)W * H; i++) {
        unsigned long long q[3];
        for (int c = 0; c < 3; c++) q[c] = (unsigned long long)(long long)quantize(rgb[i * 3 + c]);
        fprintf(f, "%llu %llu %llu \n", q[0], q[1], q[2]);
    }
    fclose(f);
    return 0;
}

/* quantised ints (as the reference's size_t) for a float buffer */
void oracle_quantize(const float *rgb, long long n, long long *out) {
    for (long long i = 0; i < n; i++) out[i] = (long long)quantize(rgb[i]);
}

#ifdef ORACLE_MAIN
/* CLI: rt_oracle scene.txt [--depth N] [--imsize W H] [--threads T]
 * Writes <scene-without-extension>.ppm like the reference and prints ray
 * counts to stderr. */
int main(int argc, char **argv) {
    if (argc < 2) {
        printf("Error: Incorrect number of arguments in input file. Please follow this formate: imsize width height\n");
        return 0;
    }
    int depth = -1, W = -1, H = -1, threads = 0;
    for (int i = 2; i < argc; i++) {
        if (!strcmp(argv[i], "--depth") && i + 1 < argc) depth = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--imsize") && i + 2 < argc) { W = atoi(argv[++i]); H = atoi(argv[++i]); }
        else if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
    }
    or_scene *S; char err[512] = {0};
    int rc = oracle_load(argv[1], &S, err, sizeof err);
    if (rc > 0) { printf("%s\n", err); return 0; }
    if (rc < 0) { fprintf(stderr, "%s\n", err); abort(); }
    if (depth >= 0) S->depth = depth;
    if (W > 0) { S->width = W; S->height = H; }
    W = S->width; H = S->height;
    int *rows = malloc(sizeof(int) * (size_t)H);
    for (int i = 0; i < H; i++) rows[i] = i;
    float *img = malloc(sizeof(float) * (size_t)W * H * 3);
    long long cnt[6];
    oracle_render_rows(S, W, H, rows, H, threads, img, cnt);
    char out[4096];
    snprintf(out, sizeof out, "%s", argv[1]);
    char *dot = strrchr(out, '.');
    if (dot) *dot = 0;
    strncat(out, ".ppm", sizeof out - strlen(out) - 1);
    oracle_write_ppm(out, img, W, H);
    fprintf(stderr, "rays prim=%lld shadow=%lld refr=%lld refl=%lld skip=%lld ub_back=%lld\n", cnt[0], cnt[1],
            cnt[2], cnt[3], cnt[4], cnt[5]);
    free(rows); free(img); oracle_free(S);
    return 0;
}
#endif
