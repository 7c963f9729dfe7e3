/*
 * ipt_oracle.c -- CPU ORACLE (test infrastructure only; see ipt_oracle.h).
 *
 * Plain-C restatement of the reference inverse path tracer.  It is NOT used
 * by the product; it is the checker the HIP kernels are compared against and
 * the timed CPU baseline of bench.py.  Build: oracle/Makefile
 * (-O2 -ffp-contract=off, so every fused multiply-add below is an explicit
 * fmaf()/fma() and nothing else is contracted).
 *
 * Canonical arithmetic, in one line per rule:
 *  - host scene precompute (vertices, normals, areas, edge planes, sampling
 *    frames, emitter CDF): unfused fp32, Eigen's expression order;
 *  - per-ray device arithmetic: dot3 = fmaf(a2,b2,fmaf(a1,b1,a0*b0)) (the
 *    contraction nvcc --fmad=true applies to Eigen's (x+y)+z reduction),
 *    cross = fmaf(a1,b2,-(a2*b1)) ..., mat·vec rows as dot chains,
 *    normalize = three IEEE divisions by sqrtf(dot3(v,v));
 *  - the reference's double-precision pow(r,0.5) is sqrt (correctly rounded);
 *    acos/sin/cos of the hemisphere angle use sin(acos(sqrt u)) = sqrtf(1-u)
 *    (1 - u in float) and cos(acos(sqrt u)) = sqrt u;
 *    sin/cos(phi) are float sinf/cosf (as the reference's float phi calls them)
 *    by one fixed fp32 reduction + polynomial, shared with the kernel.
 */
#include "ipt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------ */
/* errors                                                               */
/* ------------------------------------------------------------------ */
static char g_err[512];
static void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char *oro_last_error(void) { return g_err; }

static int g_threads = 0;
void oro_set_threads(int n) { g_threads = n; }
static int nthreads(void) {
#ifdef _OPENMP
  return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------ */
/* reference constants (scene.h:3-13, scene_basics.h:13-14, inv_scene.h:5) */
/* ------------------------------------------------------------------ */
#define P_RR 0.9f                 /* scene.h:11 */
#define MIN_DOT 1e-4              /* scene_basics.h:13 (double literal) */
#define EPSILON_T 1e-2            /* scene_basics.h:14 (double literal) */
#define PI_F ((float)M_PI)        /* Eigen `diffuse /= M_PI` converts to float */
#define INV_PI_F ((float)(1.0 / M_PI)) /* sampleNextDir returns 1/M_PI as float */

/* ------------------------------------------------------------------ */
/* cuRAND XORWOW (curand_kernel.h: curand_init / curand / curand_uniform)  */
/* call sites path_trace.cu:151-159, inv_path_trace.cu:157-165          */
/* ------------------------------------------------------------------ */
typedef struct {
  uint32_t d, v[5];
} xorwow_t;

static void xw_init(xorwow_t *s, uint64_t seed) {
  uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
  uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
  uint32_t t0 = 1099087573u * s0;
  uint32_t t1 = 2591861531u * s1;
  s->d = 6615241u + t1 + t0;
  s->v[0] = 123456789u + t0;
  s->v[1] = 362436069u ^ t0;
  s->v[2] = 521288629u + t1;
  s->v[3] = 88675123u ^ t1;
  s->v[4] = 5783321u + t0;
}
static uint32_t xw_next(xorwow_t *s) {
  uint32_t t = s->v[0] ^ (s->v[0] >> 2);
  s->v[0] = s->v[1];
  s->v[1] = s->v[2];
  s->v[2] = s->v[3];
  s->v[3] = s->v[4];
  s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
  s->d += 362437u;
  return s->v[4] + s->d;
}
/* curand_uniform: x * 2^-32 + 2^-32/2, in (0,1] */
static float xw_uniform(xorwow_t *s) {
  return (float)xw_next(s) * 2.3283064e-10f + 1.1641532e-10f;
}
float oro_uniform_at(uint64_t seed, int k) {
  xorwow_t s;
  float u = 0.f;
  xw_init(&s, seed);
  for (int i = 0; i <= k; i++) u = xw_uniform(&s);
  return u;
}

/* ------------------------------------------------------------------ */
/* deterministic double-precision elementary functions                 */
/* ------------------------------------------------------------------ */
static const double LN2_HI = 0.6931471805599453;
static const double LN2_LO = 2.3190468138462996e-17;
static const double INV_LN2 = 1.4426950408889634;

/* sinf/cosf of the float angle phi (path_trace.cu:92,96: `phi` is a float,
 * so the reference's sin(phi)/cos(phi) are CUDA's float sinf/cosf, 2 ulp)
 * in float arithmetic, operation for operation as the kernel's
 * ipt_device.h::sincos_f32: three-part Cody-Waite reduction by pi/2 (first
 * step exact for k <= 4), Cephes' degree-7 sine / degree-8 cosine on
 * |r| <= pi/4.  Exhaustively over the floats of [1e-10, 6.2832]: at most
 * 1.49 / 1.56 ulp; 76% of uniformly drawn angles correctly rounded. */
void oro_sincos(float x, float *sf, float *cf) {
  float k = rintf(x * 0x1.45f306p-1f); /* 2/pi */
  float r = fmaf(-k, 0x1.921fb6p+0f, x); /* pi/2 = C1 + C2 + C3 */
  r = fmaf(-k, -0x1.777a5cp-25f, r);
  r = fmaf(-k, -0x1.ee59dap-50f, r);
  float z = r * r;
  float p = fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f);
  p = fmaf(p, z, -1.6666654611e-1f);
  float s = fmaf(p * z, r, r);
  float q = fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f);
  q = fmaf(q, z, 4.166664568298827e-2f);
  float c = fmaf(q * z, z, fmaf(-0.5f, z, 1.0f));
  switch (((int)k) & 3) {
    case 0: *sf = s; *cf = c; break;
    case 1: *sf = c; *cf = -s; break;
    case 2: *sf = -s; *cf = -c; break;
    default: *sf = -c; *cf = s; break;
  }
}

static double bits_to_d(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static uint64_t d_to_bits(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

/* natural log for x > 0 normal: x = m 2^e, m in [sqrt(1/2), sqrt(2)),
 * log m = 2 atanh(s), s = (m-1)/(m+1), series to s^23. */
double oro_log(double x) {
  if (!(x > 0.0)) return x == 0.0 ? -INFINITY : NAN;
  if (x == INFINITY) return x;
  uint64_t b = d_to_bits(x);
  int e = (int)((b >> 52) & 0x7ff);
  if (e == 0) { /* subnormal: scale up */
    x = x * 18014398509481984.0; /* 2^54 */
    b = d_to_bits(x);
    e = (int)((b >> 52) & 0x7ff) - 54;
  }
  e -= 1023;
  double m = bits_to_d((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  if (m > 1.4142135623730951) { m *= 0.5; e += 1; }
  double s = (m - 1.0) / (m + 1.0);
  double z = s * s;
  double p = 1.0 / 23.0;
  p = fma(p, z, 1.0 / 21.0);
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  double lm = 2.0 * fma(p * z, s, s);
  double de = (double)e;
  return fma(de, LN2_HI, fma(de, LN2_LO, lm));
}
/* exp: x = k ln2 + r, |r| <= ln2/2, Taylor to r^17. */
double oro_exp(double x) {
  if (x != x) return x;
  if (x > 709.0) return INFINITY;
  if (x < -745.0) return 0.0;
  double k = rint(x * INV_LN2);
  double r = fma(-k, LN2_HI, x);
  r = fma(-k, LN2_LO, r);
  double p = 1.0 / 355687428096000.0; /* 1/17! */
  p = fma(p, r, 1.0 / 20922789888000.0);
  p = fma(p, r, 1.0 / 1307674368000.0);
  p = fma(p, r, 1.0 / 87178291200.0);
  p = fma(p, r, 1.0 / 6227020800.0);
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  int ki = (int)k;
  /* scale by 2^ki in two steps to stay in range */
  int k1 = ki / 2, k2 = ki - k1;
  double s1 = bits_to_d((uint64_t)(k1 + 1023) << 52);
  double s2 = bits_to_d((uint64_t)(k2 + 1023) << 52);
  return (p * s1) * s2;
}
static double pow_d(double x, double y) {
  if (y == 0.0) return 1.0;
  if (x == 0.0) return y > 0 ? 0.0 : INFINITY;
  return oro_exp(y * oro_log(x));
}
/* powf semantics (CUDA/C pow(float,float)) on the canonical exp/log */
float oro_powf(float x, float y) {
  if (y == 0.f) return 1.f;
  if (x == 0.f) return y > 0.f ? 0.f : INFINITY;
  if (x < 0.f) {
    if (floorf(y) != y) return NAN;
    float r = (float)pow_d(-(double)x, (double)y);
    double half = (double)y * 0.5;
    return (floor(half) != half) ? -r : r;
  }
  return (float)pow_d((double)x, (double)y);
}

/* ------------------------------------------------------------------ */
/* small fp32 vector helpers                                           */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
static v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }

/* device-side (fused, as nvcc --fmad=true) */
static float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static v3 cross_d(v3 a, v3 b) {
  return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)),
            fmaf(a.x, b.y, -(a.y * b.x)));
}
static v3 normalize_d(v3 v) {
  float n2 = dot3(v, v);
  if (n2 > 0.f) {
    float s = sqrtf(n2);
    v.x = v.x / s; v.y = v.y / s; v.z = v.z / s;
  }
  return v;
}
/* host-side (unfused, Eigen order) */
static float hdot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static v3 hcross(v3 a, v3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static v3 hnormalize(v3 v) {
  float n2 = hdot3(v, v);
  if (n2 > 0.f) {
    float s = sqrtf(n2);
    v.x = v.x / s; v.y = v.y / s; v.z = v.z / s;
  }
  return v;
}

/* ------------------------------------------------------------------ */
/* scene data (scene_basics.h:35-110, scene.h:86-173)                  */
/* ------------------------------------------------------------------ */
typedef struct {
  float diffuse[3], specular[3], emission[3], shininess;
} omat_t; /* mat_t, scene_basics.h:35-62 (fields the integrator reads) */

typedef struct {
  int idx, idxE;
  omat_t m;
  v3 v[3];
  v3 vn[3];   /* columns of Triangle::normals */
  v3 n;       /* face normal */
  v3 c;       /* centre */
  float area;
  v3 eo[3];   /* edge-plane normals (hoisted signedDistance, :497-503) */
  float ed[3];
  float R[3][3]; /* sampling frame (sampleNextDir, path_trace.cu:98-103) */
} otri_t;

typedef struct {
  int nT, nE, nO;
  int *obj_start, *obj_count; /* object ranges, object order */
  otri_t *tris;
  int *emissives; /* global triangle index per emissive */
  float *cdf, *pmf;
  float cam[4][4];
} oscene_t;

/* ------------------------------------------------------------------ */
/* number / token parsing (utils.h:70-239, 311-362, 400-444)           */
/* ------------------------------------------------------------------ */
#define IS_SPACE(x) (((x) == ' ') || ((x) == '\t'))
#define IS_DIGIT(x) ((unsigned int)((x) - '0') < 10u)
#define IS_NEW_LINE(x) (((x) == '\r') || ((x) == '\n') || ((x) == '\0'))

/* tryParseDouble, utils.h:70-200 */
static int try_parse_double(const char *s, const char *s_end, double *result) {
  if (s >= s_end) return 0;
  double mantissa = 0.0;
  int exponent = 0;
  char sign = '+', exp_sign = '+';
  const char *curr = s;
  int read = 0, end_not_reached = 0, leading_dot = 0;
  if (*curr == '+' || *curr == '-') {
    sign = *curr;
    curr++;
    if ((curr != s_end) && (*curr == '.')) leading_dot = 1;
  } else if (IS_DIGIT(*curr)) {
  } else if (*curr == '.') {
    leading_dot = 1;
  } else {
    return 0;
  }
  end_not_reached = (curr != s_end);
  if (!leading_dot) {
    while (end_not_reached && IS_DIGIT(*curr)) {
      mantissa *= 10;
      mantissa += (int)(*curr - 0x30);
      curr++;
      read++;
      end_not_reached = (curr != s_end);
    }
    if (read == 0) return 0;
  }
  if (!end_not_reached) goto assemble;
  if (*curr == '.') {
    curr++;
    read = 1;
    end_not_reached = (curr != s_end);
    while (end_not_reached && IS_DIGIT(*curr)) {
      static const double lut[] = {1.0,     0.1,      0.01,      0.001,
                                   0.0001,  0.00001,  0.000001,  0.0000001};
      mantissa += (int)(*curr - 0x30) * (read < 8 ? lut[read] : pow(10.0, -read));
      read++;
      curr++;
      end_not_reached = (curr != s_end);
    }
  } else if (*curr == 'e' || *curr == 'E') {
  } else {
    goto assemble;
  }
  if (!end_not_reached) goto assemble;
  if (*curr == 'e' || *curr == 'E') {
    curr++;
    end_not_reached = (curr != s_end);
    if (end_not_reached && (*curr == '+' || *curr == '-')) {
      exp_sign = *curr;
      curr++;
    } else if (IS_DIGIT(*curr)) {
    } else {
      return 0;
    }
    read = 0;
    end_not_reached = (curr != s_end);
    while (end_not_reached && IS_DIGIT(*curr)) {
      if (exponent > (2147483647 / 10)) return 0;
      exponent *= 10;
      exponent += (int)(*curr - 0x30);
      curr++;
      read++;
      end_not_reached = (curr != s_end);
    }
    exponent *= (exp_sign == '+' ? 1 : -1);
    if (read == 0) return 0;
  }
assemble:
  *result = (sign == '+' ? 1 : -1) *
            (exponent ? ldexp(mantissa * pow(5.0, exponent), exponent) : mantissa);
  return 1;
}
/* parseReal, utils.h:202-211 */
static float parse_real(const char **token, double dflt) {
  (*token) += strspn((*token), " \t");
  const char *end = (*token) + strcspn((*token), " \t\r");
  double val = dflt;
  try_parse_double((*token), end, &val);
  *token = end;
  return (float)val;
}
static void parse_real3(float *x, float *y, float *z, const char **token) {
  *x = parse_real(token, 0.0);
  *y = parse_real(token, 0.0);
  *z = parse_real(token, 0.0);
}
/* fixIndex / parseTriple, utils.h:287-362 */
static int fix_index(int idx, int n, int *ret) {
  if (idx > 0) { *ret = idx - 1; return 1; }
  if (idx == 0) return 0;
  *ret = n + idx;
  return 1;
}
typedef struct { int v, vt, vn; } vidx_t;
static int parse_triple(const char **token, int vsize, int vnsize, int vtsize, vidx_t *ret) {
  vidx_t vi = {-1, -1, -1};
  if (!fix_index(atoi(*token), vsize, &vi.v)) return 0;
  (*token) += strcspn((*token), "/ \t\r");
  if ((*token)[0] != '/') { *ret = vi; return 1; }
  (*token)++;
  if ((*token)[0] == '/') {
    (*token)++;
    if (!fix_index(atoi(*token), vnsize, &vi.vn)) return 0;
    (*token) += strcspn((*token), "/ \t\r");
    *ret = vi;
    return 1;
  }
  if (!fix_index(atoi(*token), vtsize, &vi.vt)) return 0;
  (*token) += strcspn((*token), "/ \t\r");
  if ((*token)[0] != '/') { *ret = vi; return 1; }
  (*token)++;
  if (!fix_index(atoi(*token), vnsize, &vi.vn)) return 0;
  (*token) += strcspn((*token), "/ \t\r");
  *ret = vi;
  return 1;
}
/* parseString, utils.h:392-399 -> copies into buf */
static void parse_string(const char **token, char *buf, size_t cap) {
  (*token) += strspn((*token), " \t");
  size_t e = strcspn((*token), " \t\r");
  size_t n = e < cap - 1 ? e : cap - 1;
  memcpy(buf, *token, n);
  buf[n] = 0;
  (*token) += e;
}

/* whole-file read; returns malloc'd NUL-terminated buffer */
static char *read_file(const char *path, size_t *len) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *b = (char *)malloc((size_t)n + 1);
  size_t got = fread(b, 1, (size_t)n, f);
  fclose(f);
  b[got] = 0;
  if (len) *len = got;
  return b;
}
/* safeGetline (utils.h:412-444): lines end at \n, \r or \r\n.  Returns the
 * next line (NUL-terminated in place) or NULL at end. */
static char *next_line(char **cursor, char *end) {
  char *p = *cursor;
  if (p >= end) return NULL;
  char *s = p;
  while (p < end && *p != '\n' && *p != '\r') p++;
  char *lend = p;
  if (p < end) {
    if (*p == '\r' && p + 1 < end && p[1] == '\n') p += 2;
    else p += 1;
  }
  *lend = 0;
  *cursor = p;
  return s;
}

/* ------------------------------------------------------------------ */
/* growable arrays                                                      */
/* ------------------------------------------------------------------ */
typedef struct { void *p; size_t n, cap, el; } vec_t;
static void *vpush(vec_t *v) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 16;
    v->p = realloc(v->p, v->cap * v->el);
  }
  return (char *)v->p + (v->n++) * v->el;
}

/* ------------------------------------------------------------------ */
/* MTL (material.h:317-367 InitMaterial, :383-772 LoadMtl)              */
/* ------------------------------------------------------------------ */
typedef struct { char name[128]; omat_t m; } named_mat_t;
static void init_material(omat_t *m) {
  for (int i = 0; i < 3; i++) m->diffuse[i] = m->specular[i] = m->emission[i] = 0.f;
  m->shininess = 1.f;
}
/* map semantics: std::map::insert keeps the FIRST index for a name */
typedef struct { vec_t mats; vec_t map_names; vec_t map_ids; } mtl_lib_t;
static int lib_lookup(mtl_lib_t *L, const char *name) {
  char(*names)[128] = (char(*)[128])L->map_names.p;
  int *ids = (int *)L->map_ids.p;
  for (size_t i = 0; i < L->map_names.n; i++)
    if (strcmp(names[i], name) == 0) return ids[i];
  return -1;
}
static void lib_insert(mtl_lib_t *L, const char *name, int id) {
  if (lib_lookup(L, name) >= 0) return;
  char *slot = (char *)vpush(&L->map_names);
  strncpy(slot, name, 127);
  slot[127] = 0;
  *(int *)vpush(&L->map_ids) = id;
}
static void load_mtl(mtl_lib_t *L, char *buf, size_t len) {
  named_mat_t cur;
  memset(&cur, 0, sizeof cur);
  init_material(&cur.m);
  char *cursor = buf, *end = buf + len, *line;
  while ((line = next_line(&cursor, end)) != NULL) {
    /* trim trailing " \t" then \n \r (material.h:404-418) */
    size_t ln = strlen(line);
    while (ln > 0 && (line[ln - 1] == ' ' || line[ln - 1] == '\t')) line[--ln] = 0;
    if (ln > 0 && line[ln - 1] == '\n') line[--ln] = 0;
    if (ln > 0 && line[ln - 1] == '\r') line[--ln] = 0;
    if (ln == 0) continue;
    const char *token = line + strspn(line, " \t");
    if (token[0] == '\0' || token[0] == '#') continue;
    if (strncmp(token, "newmtl", 6) == 0 && IS_SPACE(token[6])) {
      if (cur.name[0]) {
        lib_insert(L, cur.name, (int)L->mats.n);
        *(named_mat_t *)vpush(&L->mats) = cur;
      }
      memset(&cur, 0, sizeof cur);
      init_material(&cur.m);
      strncpy(cur.name, token + 7, 127);
      cur.name[127] = 0;
      continue;
    }
    if (token[0] == 'K' && token[1] == 'd' && IS_SPACE(token[2])) {
      token += 2;
      parse_real3(&cur.m.diffuse[0], &cur.m.diffuse[1], &cur.m.diffuse[2], &token);
      continue;
    }
    if (token[0] == 'K' && token[1] == 's' && IS_SPACE(token[2])) {
      token += 2;
      parse_real3(&cur.m.specular[0], &cur.m.specular[1], &cur.m.specular[2], &token);
      continue;
    }
    if (token[0] == 'K' && token[1] == 'e' && IS_SPACE(token[2])) {
      token += 2;
      parse_real3(&cur.m.emission[0], &cur.m.emission[1], &cur.m.emission[2], &token);
      continue;
    }
    if (token[0] == 'N' && token[1] == 's' && IS_SPACE(token[2])) {
      token += 2;
      cur.m.shininess = parse_real(&token, 0.0);
      continue;
    }
    /* every other key (Ka, Kt/Tf, Ni, illum, d, Tr, maps, PBR) leaves the
     * fields above untouched */
  }
  lib_insert(L, cur.name, (int)L->mats.n); /* flush last (material.h:765-768) */
  *(named_mat_t *)vpush(&L->mats) = cur;
}

/* ------------------------------------------------------------------ */
/* OBJ (tiny_obj_loader.h:179-583 exportGroupsToShape, :585-933 LoadObj) */
/* ------------------------------------------------------------------ */
typedef struct { vec_t v; vec_t vn; int nvt; vec_t tri; vec_t tri_mat; } objdata_t;
typedef struct { vidx_t *idx; int n; } face_t;

static void emit_tri(objdata_t *o, vidx_t a, vidx_t b, vidx_t c, int mat) {
  *(int *)vpush(&o->tri) = a.v;
  *(int *)vpush(&o->tri) = b.v;
  *(int *)vpush(&o->tri) = c.v;
  *(int *)vpush(&o->tri_mat) = mat;
}
/* pnpoly, material.h:372-381 */
static int pnpoly3(const float *vx, const float *vy, float tx, float ty) {
  int i, j, c = 0;
  for (i = 0, j = 2; i < 3; j = i++) {
    if (((vy[i] > ty) != (vy[j] > ty)) &&
        (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i]))
      c = !c;
  }
  return c;
}
static void export_group(objdata_t *o, face_t *faces, int nf, int mat) {
  const float *v = (const float *)o->v.p;
  size_t vsize = o->v.n; /* floats */
  for (int i = 0; i < nf; i++) {
    face_t *f = &faces[i];
    int npolys = f->n;
    if (npolys < 3) continue;
    if (npolys == 4) { /* quad split, tiny_obj_loader.h:205-308 */
      vidx_t i0 = f->idx[0], i1 = f->idx[1], i2 = f->idx[2], i3 = f->idx[3];
      size_t vi0 = (size_t)i0.v, vi1 = (size_t)i1.v, vi2 = (size_t)i2.v, vi3 = (size_t)i3.v;
      if (3 * vi0 + 2 >= vsize || 3 * vi1 + 2 >= vsize || 3 * vi2 + 2 >= vsize ||
          3 * vi3 + 2 >= vsize)
        continue;
      float e02x = v[vi2 * 3 + 0] - v[vi0 * 3 + 0];
      float e02y = v[vi2 * 3 + 1] - v[vi0 * 3 + 1];
      float e02z = v[vi2 * 3 + 2] - v[vi0 * 3 + 2];
      float e13x = v[vi3 * 3 + 0] - v[vi1 * 3 + 0];
      float e13y = v[vi3 * 3 + 1] - v[vi1 * 3 + 1];
      float e13z = v[vi3 * 3 + 2] - v[vi1 * 3 + 2];
      float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
      float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
      if (sqr02 < sqr13) {
        emit_tri(o, i0, i1, i2, mat);
        emit_tri(o, i0, i2, i3, mat);
      } else {
        emit_tri(o, i0, i1, i3, mat);
        emit_tri(o, i1, i2, i3, mat);
      }
      continue;
    }
    /* ear clipping, tiny_obj_loader.h:310-565 (built-in variant) */
    size_t axes[2] = {1, 2};
    for (int k = 0; k < npolys; ++k) {
      vidx_t a = f->idx[(k + 0) % npolys], b = f->idx[(k + 1) % npolys],
             c = f->idx[(k + 2) % npolys];
      size_t va = (size_t)a.v, vb = (size_t)b.v, vc = (size_t)c.v;
      if (3 * va + 2 >= vsize || 3 * vb + 2 >= vsize || 3 * vc + 2 >= vsize) continue;
      float e0x = v[vb * 3 + 0] - v[va * 3 + 0];
      float e0y = v[vb * 3 + 1] - v[va * 3 + 1];
      float e0z = v[vb * 3 + 2] - v[va * 3 + 2];
      float e1x = v[vc * 3 + 0] - v[vb * 3 + 0];
      float e1y = v[vc * 3 + 1] - v[vb * 3 + 1];
      float e1z = v[vc * 3 + 2] - v[vb * 3 + 2];
      float cx = fabsf(e0y * e1z - e0z * e1y);
      float cy = fabsf(e0z * e1x - e0x * e1z);
      float cz = fabsf(e0x * e1y - e0y * e1x);
      const float eps = FLT_EPSILON;
      if (cx > eps || cy > eps || cz > eps) {
        if (!(cx > cy && cx > cz)) {
          axes[0] = 0;
          if (cz > cx && cz > cy) axes[1] = 1;
        }
        break;
      }
    }
    int rn = npolys;
    vidx_t *rem = (vidx_t *)malloc(sizeof(vidx_t) * (size_t)npolys);
    memcpy(rem, f->idx, sizeof(vidx_t) * (size_t)npolys);
    size_t guess = 0;
    size_t remaining_iter = (size_t)npolys;
    size_t prev_rem = (size_t)npolys;
    vidx_t ind[3];
    float vx[3], vy[3];
    while (rn > 3 && remaining_iter > 0) {
      size_t np = (size_t)rn;
      if (guess >= np) guess -= np;
      if (prev_rem != np) {
        prev_rem = np;
        remaining_iter = np;
      } else {
        remaining_iter--;
      }
      for (size_t k = 0; k < 3; k++) {
        ind[k] = rem[(guess + k) % np];
        size_t vi = (size_t)ind[k].v;
        if ((vi * 3 + axes[0]) >= vsize || (vi * 3 + axes[1]) >= vsize) {
          vx[k] = 0.f;
          vy[k] = 0.f;
        } else {
          vx[k] = v[vi * 3 + axes[0]];
          vy[k] = v[vi * 3 + axes[1]];
        }
      }
      float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0];
      float e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
      float cross = e0x * e1y - e0y * e1x;
      float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
      if (cross * area < 0.f) {
        guess += 1;
        continue;
      }
      int overlap = 0;
      for (size_t other = 3; other < np; ++other) {
        size_t idx = (guess + other) % np;
        if (idx >= (size_t)rn) continue;
        size_t ovi = (size_t)rem[idx].v;
        if ((ovi * 3 + axes[0]) >= vsize || (ovi * 3 + axes[1]) >= vsize) continue;
        float tx = v[ovi * 3 + axes[0]], ty = v[ovi * 3 + axes[1]];
        if (pnpoly3(vx, vy, tx, ty)) {
          overlap = 1;
          break;
        }
      }
      if (overlap) {
        guess += 1;
        continue;
      }
      emit_tri(o, ind[0], ind[1], ind[2], mat);
      size_t removed = (guess + 1) % np;
      while (removed + 1 < np) {
        rem[removed] = rem[removed + 1];
        removed += 1;
      }
      rn--;
    }
    if (rn == 3) emit_tri(o, rem[0], rem[1], rem[2], mat);
    free(rem);
  }
}

/* LoadObj (tiny_obj_loader.h:585-933) with the scene-supplied MTL stream
 * (scene_basics.h:221-233): mtllib consults `mtlbuf` (NULL = stream in
 * error state -> no materials). */
static int load_obj(char *buf, size_t len, char *mtlbuf, size_t mtllen, objdata_t *o,
                    mtl_lib_t *L) {
  vec_t faces = {0, 0, 0, sizeof(face_t)};
  int material = -1;
  int mtl_consumed = 0;
  char *cursor = buf, *end = buf + len, *line;
  while ((line = next_line(&cursor, end)) != NULL) {
    size_t ln = strlen(line);
    if (ln > 0 && line[ln - 1] == '\n') line[--ln] = 0;
    if (ln > 0 && line[ln - 1] == '\r') line[--ln] = 0;
    if (ln == 0) continue;
    const char *token = line + strspn(line, " \t");
    if (token[0] == '\0' || token[0] == '#') continue;
    if (token[0] == 'v' && IS_SPACE(token[1])) {
      token += 2;
      float x = parse_real(&token, 0.0), y = parse_real(&token, 0.0),
            z = parse_real(&token, 0.0);
      *(float *)vpush(&o->v) = x;
      *(float *)vpush(&o->v) = y;
      *(float *)vpush(&o->v) = z;
      continue;
    }
    if (token[0] == 'v' && token[1] == 'n' && IS_SPACE(token[2])) {
      token += 3;
      float x, y, z;
      parse_real3(&x, &y, &z, &token);
      *(float *)vpush(&o->vn) = x;
      *(float *)vpush(&o->vn) = y;
      *(float *)vpush(&o->vn) = z;
      continue;
    }
    if (token[0] == 'v' && token[1] == 't' && IS_SPACE(token[2])) {
      o->nvt++;
      continue;
    }
    if (token[0] == 'f' && IS_SPACE(token[1])) {
      token += 2;
      token += strspn(token, " \t");
      vec_t fi = {0, 0, 0, sizeof(vidx_t)};
      while (!IS_NEW_LINE(token[0])) {
        vidx_t vi;
        if (!parse_triple(&token, (int)(o->v.n / 3), (int)(o->vn.n / 3), o->nvt, &vi)) {
          set_err("failed to parse `f' line (zero face index)");
          free(fi.p);
          return 0;
        }
        *(vidx_t *)vpush(&fi) = vi;
        token += strspn(token, " \t\r");
      }
      face_t *fc = (face_t *)vpush(&faces);
      fc->idx = (vidx_t *)fi.p;
      fc->n = (int)fi.n;
      continue;
    }
    if (strncmp(token, "usemtl", 6) == 0) {
      token += 6;
      char name[128];
      parse_string(&token, name, sizeof name);
      int nid = lib_lookup(L, name);
      if (nid != material) {
        export_group(o, (face_t *)faces.p, (int)faces.n, material);
        for (size_t i = 0; i < faces.n; i++) free(((face_t *)faces.p)[i].idx);
        faces.n = 0;
        material = nid;
      }
      continue;
    }
    if (strncmp(token, "mtllib", 6) == 0 && IS_SPACE(token[6])) {
      /* MaterialStreamReader ignores the filename and reads the scene-file
       * stream; a second mtllib finds the stream at EOF. */
      if (mtlbuf && !mtl_consumed) load_mtl(L, mtlbuf, mtllen);
      mtl_consumed = 1;
      continue;
    }
    if ((token[0] == 'g' || token[0] == 'o') && IS_SPACE(token[1])) {
      export_group(o, (face_t *)faces.p, (int)faces.n, material);
      for (size_t i = 0; i < faces.n; i++) free(((face_t *)faces.p)[i].idx);
      faces.n = 0;
      continue;
    }
  }
  export_group(o, (face_t *)faces.p, (int)faces.n, material);
  for (size_t i = 0; i < faces.n; i++) free(((face_t *)faces.p)[i].idx);
  free(faces.p);
  return 1;
}

/* ------------------------------------------------------------------ */
/* Mesh::Mesh / ParseFromString / Triangle (scene_basics.h:74-289)      */
/* ------------------------------------------------------------------ */
/* Eigen AngleAxis::toRotationMatrix */
static void angle_axis(float angle, v3 axis, float R[3][3]) {
  float s = sinf(angle), c = cosf(angle);
  v3 sa = mk(s * axis.x, s * axis.y, s * axis.z);
  float omc = 1.f - c;
  v3 ca = mk(omc * axis.x, omc * axis.y, omc * axis.z);
  float tmp;
  tmp = ca.x * axis.y;
  R[0][1] = tmp - sa.z;
  R[1][0] = tmp + sa.z;
  tmp = ca.x * axis.z;
  R[0][2] = tmp + sa.y;
  R[2][0] = tmp - sa.y;
  tmp = ca.y * axis.z;
  R[1][2] = tmp - sa.x;
  R[2][1] = tmp + sa.x;
  R[0][0] = ca.x * axis.x + c;
  R[1][1] = ca.y * axis.y + c;
  R[2][2] = ca.z * axis.z + c;
}
/* Eigen Quaternion::setFromTwoVectors((0,0,1), n).toRotationMatrix() */
static void frame_from_normal(v3 n, float R[3][3]) {
  if (n.z == -1.f) { /* path_trace.cu:99-100 */
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i][j] = (i == j) ? -1.f : 0.f;
    return;
  }
  v3 v0 = mk(0.f, 0.f, 1.f);
  v3 v1 = hnormalize(n);
  float c = hdot3(v1, v0);
  float qx, qy, qz, qw;
  if (c < -1.f + 1e-5f) {
    /* Eigen takes an SVD null-space axis here; never reached by shipped
     * assets.  We take the normalised cross product. */
    c = c > -1.f ? c : -1.f;
    v3 ax = hcross(v0, v1);
    if (hdot3(ax, ax) > 0.f) ax = hnormalize(ax);
    else ax = mk(1.f, 0.f, 0.f);
    float w2 = (1.f + c) * 0.5f;
    qw = sqrtf(w2);
    float sv = sqrtf(1.f - w2);
    qx = ax.x * sv; qy = ax.y * sv; qz = ax.z * sv;
  } else {
    v3 axis = hcross(v0, v1);
    float s = sqrtf((1.f + c) * 2.f);
    float invs = 1.f / s;
    qx = axis.x * invs; qy = axis.y * invs; qz = axis.z * invs;
    qw = s * 0.5f;
  }
  float tx = 2.f * qx, ty = 2.f * qy, tz = 2.f * qz;
  float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  R[0][0] = 1.f - (tyy + tzz);
  R[0][1] = txy - twz;
  R[0][2] = txz + twy;
  R[1][0] = txy + twz;
  R[1][1] = 1.f - (txx + tzz);
  R[1][2] = tyz - twx;
  R[2][0] = txz - twy;
  R[2][1] = tyz + twx;
  R[2][2] = 1.f - (txx + tyy);
}
/* Triangle::Triangle, scene_basics.h:74-96, plus the hoisted per-triangle
 * constants of signedDistance (:497-503) and sampleNextDir (path_trace.cu:98-103) */
static void build_triangle(otri_t *t, int i, const omat_t *m, v3 a, v3 b, v3 c, const v3 *ns) {
  t->idx = i;
  t->idxE = -1;
  t->m = *m;
  t->v[0] = a; t->v[1] = b; t->v[2] = c;
  v3 ctr = mk(0.f, 0.f, 0.f);
  for (int j = 0; j < 3; j++) {
    ctr.x = ctr.x + t->v[j].x / 3.f;
    ctr.y = ctr.y + t->v[j].y / 3.f;
    ctr.z = ctr.z + t->v[j].z / 3.f;
  }
  t->c = ctr;
  v3 e0 = sub(t->v[1], t->v[0]);
  v3 e1 = sub(t->v[2], t->v[1]);
  v3 n = hcross(e0, e1);
  t->area = sqrtf(hdot3(n, n)) / 2.f;
  n = hnormalize(n);
  t->n = n;
  for (int j = 0; j < 3; j++) t->vn[j] = ns ? ns[j] : n;
  for (int j = 0; j < 3; j++) {
    v3 s0 = t->v[j], s1 = t->v[(j + 1) % 3];
    v3 out = hnormalize(hcross(sub(s1, s0), n));
    t->eo[j] = out;
    t->ed[j] = -hdot3(out, add(s1, s0)) / 2.f;
  }
  frame_from_normal(n, t->R);
}

static int build_mesh(const float *pos, const float *ori, const float *scl, const char *objp,
                      const char *mtlp, vec_t *tris, int *n_out) {
  /* Transform, scene_basics.h:148-157 */
  v3 o = mk(ori[0], ori[1], ori[2]);
  float angle = sqrtf(hdot3(o, o));
  o = hnormalize(o);
  float R[3][3];
  angle_axis(angle, o, R);
  float Lm[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Lm[i][j] = R[i][j] * scl[j];
  float tr[3] = {pos[0], pos[1], pos[2]};

  size_t olen = 0;
  char *obuf = read_file(objp, &olen);
  if (!obuf) {
    set_err("Object File was not able to be opened: %s", objp);
    return 0;
  }
  int in_string = mtlp[0] == '*';
  size_t mlen = 0;
  char *mbuf = in_string ? NULL : read_file(mtlp, &mlen);
  objdata_t od;
  memset(&od, 0, sizeof od);
  od.v.el = od.vn.el = sizeof(float);
  od.tri.el = od.tri_mat.el = sizeof(int);
  mtl_lib_t L;
  memset(&L, 0, sizeof L);
  L.mats.el = sizeof(named_mat_t);
  L.map_names.el = 128;
  L.map_ids.el = sizeof(int);
  int ok = load_obj(obuf, olen, mbuf, mlen, &od, &L);
  free(obuf);
  free(mbuf);
  if (!ok) return 0;

  /* inline material, scene_basics.h:249-268 */
  omat_t rand_mat;
  init_material(&rand_mat);
  if (in_string) {
    size_t ml = strlen(mtlp);
    char *s = (char *)malloc(ml + 1);
    size_t sl = ml >= 2 ? ml - 2 : 0;
    memcpy(s, mtlp + 1, sl);
    s[sl] = 0;
    char *p = s;
    while (p && *p) {
      char *nl = strchr(p, '\n');
      if (nl) *nl = 0;
      const char *token = p;
      if (strlen(token) >= 3 && token[0] == 'K' && IS_SPACE(token[2])) {
        char k = token[1];
        token += 2;
        float r, g, b;
        parse_real3(&r, &g, &b, &token);
        if (k == 'd') {
          rand_mat.diffuse[0] = r;
          rand_mat.diffuse[1] = g;
          rand_mat.diffuse[2] = b;
        }
      }
      p = nl ? nl + 1 : NULL;
    }
    free(s);
  }
  /* transform vertices and normals (scene_basics.h:235-243) */
  size_t nv = od.v.n / 3, nn = od.vn.n / 3;
  v3 *vs = (v3 *)malloc(sizeof(v3) * (nv ? nv : 1));
  v3 *vns = (v3 *)malloc(sizeof(v3) * (nn ? nn : 1));
  const float *vr = (const float *)od.v.p;
  for (size_t i = 0; i < nv; i++) {
    float x = vr[3 * i], y = vr[3 * i + 1], z = vr[3 * i + 2];
    float r[3];
    for (int k = 0; k < 3; k++) r[k] = ((Lm[k][0] * x + Lm[k][1] * y) + Lm[k][2] * z) + tr[k];
    vs[i] = mk(r[0], r[1], r[2]);
  }
  /* T.linear().transpose().inverse() via Eigen's 3x3 cofactor inverse */
  float A[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) A[i][j] = Lm[j][i];
#define COF(i, j)                                                              \
  (A[((i) + 1) % 3][((j) + 1) % 3] * A[((i) + 2) % 3][((j) + 2) % 3] -        \
   A[((i) + 1) % 3][((j) + 2) % 3] * A[((i) + 2) % 3][((j) + 1) % 3])
  float c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
  float det = (c00 * A[0][0] + c10 * A[1][0]) + c20 * A[2][0];
  float invdet = 1.f / det;
  float T2[3][3];
  T2[0][0] = c00 * invdet; T2[0][1] = c10 * invdet; T2[0][2] = c20 * invdet;
  T2[1][0] = COF(0, 1) * invdet; T2[1][1] = COF(1, 1) * invdet; T2[1][2] = COF(2, 1) * invdet;
  T2[2][0] = COF(0, 2) * invdet; T2[2][1] = COF(1, 2) * invdet; T2[2][2] = COF(2, 2) * invdet;
#undef COF
  const float *nr = (const float *)od.vn.p;
  for (size_t i = 0; i < nn; i++) {
    float x = nr[3 * i], y = nr[3 * i + 1], z = nr[3 * i + 2];
    float r[3];
    for (int k = 0; k < 3; k++) r[k] = (T2[k][0] * x + T2[k][1] * y) + T2[k][2] * z;
    vns[i] = mk(r[0], r[1], r[2]);
  }
  /* faces -> triangles (scene_basics.h:168-193) */
  size_t nf = od.tri_mat.n;
  const int *fi = (const int *)od.tri.p;
  const int *fm = (const int *)od.tri_mat.p;
  named_mat_t *mats = (named_mat_t *)L.mats.p;
  for (size_t i = 0; i < nf; i++) {
    int a = fi[3 * i], b = fi[3 * i + 1], c = fi[3 * i + 2];
    if (a < 0 || b < 0 || c < 0 || (size_t)a >= nv || (size_t)b >= nv || (size_t)c >= nv) {
      set_err("face %zu references a vertex out of range", i);
      return 0;
    }
    const omat_t *m = (fm[i] != -1) ? &mats[fm[i]].m : &rand_mat;
    v3 ns3[3];
    const v3 *nsp = NULL;
    if (nn == nv) {
      ns3[0] = vns[a]; ns3[1] = vns[b]; ns3[2] = vns[c];
      nsp = ns3;
    }
    otri_t *t = (otri_t *)vpush(tris);
    build_triangle(t, (int)i, m, vs[a], vs[b], vs[c], nsp);
  }
  *n_out = (int)nf;
  free(vs); free(vns);
  free(od.v.p); free(od.vn.p); free(od.tri.p); free(od.tri_mat.p);
  free(L.mats.p); free(L.map_names.p); free(L.map_ids.p);
  return 1;
}

/* Camera (scene.h:15-84) with the default CameraParams_t(true) */
static void camera_matrix(float M[4][4]) {
  v3 pos = mk(0.f, 0.f, 0.f), look = mk(0.f, 0.f, 1.f), up = mk(0.f, 1.f, 0.f);
  float ha = (float)(M_PI * (double)90.f / (double)360.f);
  float ar = 1.f;
  v3 dir = hnormalize(look);
  up = hnormalize(up);
  v3 f = hnormalize(dir);
  v3 s = hnormalize(hcross(f, up));
  v3 u = hnormalize(hcross(s, f));
  float V[4][4] = {{s.x, s.y, s.z, -hdot3(s, pos)},
                   {u.x, u.y, u.z, -hdot3(u, pos)},
                   {f.x, f.y, f.z, -hdot3(f, pos)},
                   {0.f, 0.f, 0.f, 1.f}};
  float S[4][4] = {{tanf(ha), 0, 0, 0}, {0, tanf(ha * ar), 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      M[i][j] = ((S[i][0] * V[j][0] + S[i][1] * V[j][1]) + S[i][2] * V[j][2]) + S[i][3] * V[j][3];
}

void *oro_load_scene(int n, const float *poss, const float *oris, const float *scls,
                     const char **obj_files, const char **mtl_files) {
  oscene_t *sc = (oscene_t *)calloc(1, sizeof(oscene_t));
  vec_t tris = {0, 0, 0, sizeof(otri_t)};
  sc->nO = n;
  sc->obj_start = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
  sc->obj_count = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
  for (int o = 0; o < n; o++) {
    int cnt = 0;
    size_t before = tris.n;
    if (!build_mesh(poss + 3 * o, oris + 3 * o, scls + 3 * o, obj_files[o], mtl_files[o],
                    &tris, &cnt)) {
      free(tris.p);
      free(sc->obj_start);
      free(sc->obj_count);
      free(sc);
      return NULL;
    }
    sc->obj_start[o] = (int)before;
    sc->obj_count[o] = cnt;
  }
  sc->tris = (otri_t *)tris.p;
  sc->nT = (int)tris.n;
  /* setOffsets + emissive list (scene.h:96-113, scene_basics.h:183-187,467-474) */
  int ne = 0;
  for (int i = 0; i < sc->nT; i++) {
    otri_t *t = &sc->tris[i];
    t->idx = i;
    if (t->m.emission[0] > 0.f || t->m.emission[1] > 0.f || t->m.emission[2] > 0.f) {
      t->idxE = ne++;
    }
  }
  sc->nE = ne;
  sc->emissives = (int *)malloc(sizeof(int) * (size_t)(ne ? ne : 1));
  sc->cdf = (float *)malloc(sizeof(float) * (size_t)(ne ? ne : 1));
  sc->pmf = (float *)malloc(sizeof(float) * (size_t)(ne ? ne : 1));
  for (int i = 0; i < sc->nT; i++)
    if (sc->tris[i].idxE >= 0) sc->emissives[sc->tris[i].idxE] = i;
  /* emitter CDF, path_trace.cu:39-51 */
  float area_sum = 0.f;
  for (int i = 0; i < ne; i++) area_sum += sc->tris[sc->emissives[i]].area;
  float pc = 0.f;
  for (int i = 0; i < ne; i++) {
    float p = sc->tris[sc->emissives[i]].area / area_sum;
    pc += p;
    sc->cdf[i] = pc;
    sc->pmf[i] = p;
  }
  camera_matrix(sc->cam);
  return sc;
}

void oro_free_scene(void *p) {
  oscene_t *sc = (oscene_t *)p;
  if (!sc) return;
  free(sc->tris); free(sc->emissives); free(sc->cdf); free(sc->pmf);
  free(sc->obj_start); free(sc->obj_count);
  free(sc);
}
int oro_num_triangles(void *p) { return ((oscene_t *)p)->nT; }
int oro_num_emissives(void *p) { return ((oscene_t *)p)->nE; }
void oro_camera_matrix(void *p, float *out16) {
  oscene_t *sc = (oscene_t *)p;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) out16[i * 4 + j] = sc->cam[i][j];
}
void oro_export_triangles(void *p, float *out) {
  oscene_t *sc = (oscene_t *)p;
  for (int i = 0; i < sc->nT; i++) {
    otri_t *t = &sc->tris[i];
    float *o = out + (size_t)i * ORO_TRI_STRIDE;
    for (int j = 0; j < 3; j++) {
      o[3 * j] = t->v[j].x; o[3 * j + 1] = t->v[j].y; o[3 * j + 2] = t->v[j].z;
      o[9 + 3 * j] = t->vn[j].x; o[10 + 3 * j] = t->vn[j].y; o[11 + 3 * j] = t->vn[j].z;
    }
    o[18] = t->n.x; o[19] = t->n.y; o[20] = t->n.z;
    o[21] = t->c.x; o[22] = t->c.y; o[23] = t->c.z;
    o[24] = t->area;
    for (int j = 0; j < 3; j++) {
      o[25 + j] = t->m.diffuse[j];
      o[28 + j] = t->m.specular[j];
      o[31 + j] = t->m.emission[j];
    }
    o[34] = t->m.shininess;
    for (int j = 0; j < 3; j++) {
      o[35 + 4 * j] = t->eo[j].x; o[36 + 4 * j] = t->eo[j].y;
      o[37 + 4 * j] = t->eo[j].z; o[38 + 4 * j] = t->ed[j];
    }
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) o[47 + 3 * a + b] = t->R[a][b];
    o[56] = (float)t->idxE;
  }
}
/* Scene::getMaterials / setMaterials (scene.h:145-162) */
void oro_get_materials(void *p, float *out) {
  oscene_t *sc = (oscene_t *)p;
  for (int i = 0; i < sc->nT; i++)
    for (int j = 0; j < 3; j++) out[3 * i + j] = sc->tris[i].m.diffuse[j];
}
void oro_set_materials(void *p, const float *in) {
  oscene_t *sc = (oscene_t *)p;
  for (int i = 0; i < sc->nT; i++)
    for (int j = 0; j < 3; j++) sc->tris[i].m.diffuse[j] = in[3 * i + j];
}

/* ------------------------------------------------------------------ */
/* ray queries                                                          */
/* ------------------------------------------------------------------ */
typedef struct { v3 p, d; } ray_t;
typedef struct { float t; int tri; } hit_t;

/* BVH::getIntersection (bvh.h:37-107) over a single leaf ->
 * Object::getIntersection (scene_basics.h:426-459) per object, objects in
 * load order; strict '<' keeps the first of equal-t hits. */
static hit_t intersect(const oscene_t *sc, ray_t r) {
  hit_t best = {INFINITY, -1};
  for (int o = 0; o < sc->nO; o++) {
    hit_t cur = {INFINITY, -1};
    for (int k = 0; k < sc->obj_count[o]; k++) {
      int i = sc->obj_start[o] + k;
      const otri_t *t = &sc->tris[i];
      float denom = dot3(t->n, r.d);
      if ((double)fabsf(denom) < MIN_DOT) continue;
      float tt = dot3(sub(r.p, t->c), t->n) / -denom;
      if ((double)tt < EPSILON_T || tt >= cur.t) continue;
      v3 q = mk(fmaf(r.d.x, tt, r.p.x), fmaf(r.d.y, tt, r.p.y), fmaf(r.d.z, tt, r.p.z));
      int inside = 1;
      for (int j = 0; j < 3; j++) {
        float sd = fmaf(q.z, t->eo[j].z, fmaf(q.y, t->eo[j].y, fmaf(q.x, t->eo[j].x, t->ed[j])));
        if (sd > 0.f) { inside = 0; break; }
      }
      if (!inside) continue;
      cur.t = tt;
      cur.tri = i;
    }
    if (cur.tri >= 0 && cur.t < best.t) best = cur;
  }
  return best;
}
/* Closest hit of caller rays (the parity anchor of the kernels' BVH). */
int oro_closest_hit(void *p, int64_t n, const float *org, const float *dir, float *t, int *idx) {
  const oscene_t *sc = (const oscene_t *)p;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) {
    ray_t r;
    r.p = mk(org[3 * i], org[3 * i + 1], org[3 * i + 2]);
    r.d = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    hit_t h = intersect(sc, r);
    t[i] = h.t;
    idx[i] = h.tri;
  }
  return 0;
}
/* The single-triangle test of intersect() without the best-t condition:
 * t_out[i] = the t at which triangle i accepts the ray, NaN if it rejects.
 * Test infrastructure for the BVH's acceptance-region bound. */
int oro_hit_each(void *p, const float *org, const float *dir, float *t_out) {
  const oscene_t *sc = (const oscene_t *)p;
  ray_t r;
  r.p = mk(org[0], org[1], org[2]);
  r.d = mk(dir[0], dir[1], dir[2]);
  for (int i = 0; i < sc->nT; i++) {
    const otri_t *t = &sc->tris[i];
    t_out[i] = NAN;
    float denom = dot3(t->n, r.d);
    if ((double)fabsf(denom) < MIN_DOT) continue;
    float tt = dot3(sub(r.p, t->c), t->n) / -denom;
    if ((double)tt < EPSILON_T) continue;
    v3 q = mk(fmaf(r.d.x, tt, r.p.x), fmaf(r.d.y, tt, r.p.y), fmaf(r.d.z, tt, r.p.z));
    int inside = 1;
    for (int j = 0; j < 3; j++) {
      float sd = fmaf(q.z, t->eo[j].z, fmaf(q.y, t->eo[j].y, fmaf(q.x, t->eo[j].x, t->ed[j])));
      if (sd > 0.f) { inside = 0; break; }
    }
    if (inside) t_out[i] = tt;
  }
  return 0;
}
static v3 hit_point(ray_t r, float t) {
  return mk(fmaf(r.d.x, t, r.p.x), fmaf(r.d.y, t, r.p.y), fmaf(r.d.z, t, r.p.z));
}
/* Triangle::getNormal (scene_basics.h:100-109) */
static v3 get_normal(const otri_t *t, v3 q) {
  float w[3];
  for (int i = 0; i < 3; i++) {
    v3 a = sub(t->v[(i + 1) % 3], q), b = sub(t->v[(i + 2) % 3], q);
    v3 cr = cross_d(a, b);
    w[i] = (0.5f * sqrtf(dot3(cr, cr))) / t->area;
  }
  v3 n = mk(fmaf(t->vn[2].x, w[2], fmaf(t->vn[1].x, w[1], t->vn[0].x * w[0])),
            fmaf(t->vn[2].y, w[2], fmaf(t->vn[1].y, w[1], t->vn[0].y * w[0])),
            fmaf(t->vn[2].z, w[2], fmaf(t->vn[1].z, w[1], t->vn[0].z * w[0])));
  return normalize_d(n);
}
/* camera ray, path_trace.cu:150-165 + Ray::transform scene_basics.h:307-319 */
static ray_t camera_ray(const oscene_t *sc, xorwow_t *st, int r, int c, int W, int H) {
  float u0 = xw_uniform(st), u1 = xw_uniform(st);
  float x = 2.f * ((float)c + u0) / (float)W - 1.f;
  float y = 1.f - 2.f * ((float)r + u1) / (float)H;
  v3 d = normalize_d(mk(x, y, 1.f));
  const float(*M)[4] = sc->cam;
  float p4[4] = {0.f, 0.f, 0.f, 1.f}, d4[4] = {d.x, d.y, d.z, 0.f}, pr[3], dr[3];
  for (int i = 0; i < 3; i++) {
    pr[i] = fmaf(M[i][3], p4[3], fmaf(M[i][2], p4[2], fmaf(M[i][1], p4[1], M[i][0] * p4[0])));
    dr[i] = fmaf(M[i][3], d4[3], fmaf(M[i][2], d4[2], fmaf(M[i][1], d4[1], M[i][0] * d4[0])));
  }
  ray_t ray;
  ray.p = mk(pr[0], pr[1], pr[2]);
  ray.d = normalize_d(mk(dr[0], dr[1], dr[2]));
  return ray;
}
/* emitter choice, path_trace.cu:39-51 (clamped if rounding leaves cdf<u) */
static int pick_emitter(const oscene_t *sc, float u) {
  int idx = 0;
  for (int i = 0; i < sc->nE; i++) {
    if (sc->cdf[i] >= u) break;
    idx++;
  }
  return idx < sc->nE ? idx : sc->nE - 1;
}
static int is_specular(const omat_t *m) {
  return (m->specular[0] != 0.f || m->specular[1] != 0.f || m->specular[2] != 0.f) &&
         m->shininess != 0.f;
}
/* Phong lobe coefficient of BSDF (path_trace.cu:19-22) */
static float phong_coeff(const omat_t *m, v3 nrm, v3 w, v3 wi) {
  float dn = dot3(nrm, wi);
  v3 refl = mk(fmaf(2.f * dn, nrm.x, -wi.x), fmaf(2.f * dn, nrm.y, -wi.y),
               fmaf(2.f * dn, nrm.z, -wi.z));
  float pw = oro_powf(dot3(refl, w), m->shininess);
  float mx = pw > 0.f ? pw : 0.f; /* fmaxf(pw, 0): NaN -> 0 */
  return (float)((((double)(m->shininess + 2.f)) / 2.0 / M_PI) * (double)mx);
}

typedef struct {
  int ok;        /* NEE found the sampled emitter */
  int emitter;   /* global tri index */
  float ct, ctp, ts;
  float s;       /* cos*cos'/t^2/p_t as float (forward) */
  double g;      /* cos*cos'/t^2 /p_t in double, before the float cast */
  v3 toLight;
} nee_t;

/* geometry of directLighting (path_trace.cu:30-86 / inv_path_trace.cu:16-65):
 * consumes 3 draws when nE > 0. `wct` scales cos(theta) first (graph:
 * prev_weight*cos_theta), 1.f for the forward integrator. */
static nee_t nee_geometry(const oscene_t *sc, const otri_t *tri, v3 q, v3 nh, float wct,
                          xorwow_t *st, int64_t *casts) {
  nee_t r;
  memset(&r, 0, sizeof r);
  r.emitter = -1;
  if (sc->nE == 0) return r;
  float u = xw_uniform(st);
  int ie = pick_emitter(sc, u);
  float p_t = sc->pmf[ie];
  const otri_t *te = &sc->tris[sc->emissives[ie]];
  float r1 = xw_uniform(st), r2 = xw_uniform(st);
  double sq = sqrt((double)r1);
  float a = (float)(1.0 - sq);
  float b = (float)(sq * (double)(1.f - r2));
  float c = (float)((double)r2 * sq);
  v3 pt = mk(fmaf(c, te->v[2].x, fmaf(b, te->v[1].x, a * te->v[0].x)),
             fmaf(c, te->v[2].y, fmaf(b, te->v[1].y, a * te->v[0].y)),
             fmaf(c, te->v[2].z, fmaf(b, te->v[1].z, a * te->v[0].z)));
  v3 tl = normalize_d(sub(pt, q));
  r.toLight = tl;
  float ct = dot3(nh, tl);
  if (ct < 0.f) return r;
  ray_t lr = {q, tl};
  if (casts) (*casts)++;
  hit_t h = intersect(sc, lr);
  if (h.tri < 0) return r;
  if (h.tri != sc->emissives[ie]) return r; /* checked before cos' (both return 0) */
  v3 qs = hit_point(lr, h.t);
  v3 ne = get_normal(te, qs);
  float ctp = -dot3(ne, tl);
  if (ctp < 0.f) return r;
  r.ok = 1;
  r.emitter = sc->emissives[ie];
  r.ct = ct;
  r.ctp = ctp;
  r.ts = h.t;
  double td = (double)h.t;
  r.g = ((double)((wct * ct) * ctp) / (td * td)) / (double)p_t;
  r.s = (float)r.g;
  (void)tri;
  return r;
}

/* sampleNextDir (path_trace.cu:91-109): 2 draws */
static v3 sample_dir(const otri_t *tri, int spec, float shin, float *psamp, xorwow_t *st) {
  float uphi = xw_uniform(st);
  float phi = (float)(2 * M_PI * (double)uphi);
  float ut = xw_uniform(st);
  float ct, snt;
  if (!spec) {
    ct = (float)sqrt((double)ut);
    snt = sqrtf(1.0f - ut); /* sin(acos(sqrt u)) = sqrt(1 - u), from the float 1 - u */
    *psamp = INV_PI_F;
  } else {
    double e = 1.0 / ((double)shin + 1.0);
    double cd = pow_d((double)ut, e);
    ct = (float)cd;
    snt = (float)sqrt(1.0 - cd * cd);
    *psamp = oro_powf((shin + 1.f) * ct, shin);
  }
  float sp, cp;
  oro_sincos(phi, &sp, &cp);
  v3 h = mk(snt * cp, snt * sp, ct);
  const float(*R)[3] = tri->R;
  v3 nd = mk(fmaf(R[0][2], h.z, fmaf(R[0][1], h.y, R[0][0] * h.x)),
             fmaf(R[1][2], h.z, fmaf(R[1][1], h.y, R[1][0] * h.x)),
             fmaf(R[2][2], h.z, fmaf(R[2][1], h.y, R[2][0] * h.x)));
  return normalize_d(nd);
}

/* per-vertex record for the adjoint */
typedef struct {
  int tri;
  float lo[3];     /* Ke * s (0 if NEE failed) */
  float specd;     /* direct Phong coefficient (0 if none) */
  float coeff;     /* cos/p/p_RR (continued vertices) */
  float speci;     /* indirect Phong coefficient */
} vrec_t;

/* One forward sample: renderSample + radiance, path_trace.cu:111-184.
 * rec (nullable, capacity max_bounces+1) receives the path vertices for the
 * adjoint; *nrec their count, *esc whether the path ended by a miss. */
static void trace_forward(const oscene_t *sc, int W, int H, int spp, int max_bounces,
                          uint64_t seed, int64_t gidx, float L[3], int64_t *casts,
                          vrec_t *rec, int *nrec, int *esc) {
  xorwow_t st;
  xw_init(&st, seed + (uint64_t)gidx);
  int64_t pix = gidx / spp;
  int r = (int)(pix / W), c = (int)(pix % W);
  ray_t ray = camera_ray(sc, &st, r, c, W, H);
  float Le[3] = {0, 0, 0}, Ld[3] = {0, 0, 0}, M[3] = {1, 1, 1};
  L[0] = L[1] = L[2] = 0.f;
  int k = 0, n = 0;
  if (esc) *esc = 0;
  for (;;) {
    float Mp[3] = {M[0], M[1], M[2]};
    int cont = 0;
    /* radiance() */
    if (casts) (*casts)++;
    hit_t h = intersect(sc, ray);
    if (h.tri < 0) {
      if (esc && k > 0) *esc = 1;
    } else {
      const otri_t *tri = &sc->tris[h.tri];
      v3 q = hit_point(ray, h.t);
      if (k == 0)
        for (int i = 0; i < 3; i++) Le[i] = tri->m.emission[i];
      v3 nh = get_normal(tri, q);
      nee_t ne = nee_geometry(sc, tri, q, nh, 1.f, &st, casts);
      int spec = is_specular(&tri->m);
      float specd = 0.f;
      if (ne.ok) {
        const otri_t *te = &sc->tris[ne.emitter];
        if (tri->m.specular[0] != 0.f || tri->m.specular[1] != 0.f || tri->m.specular[2] != 0.f)
          specd = phong_coeff(&tri->m, nh, ray.d, ne.toLight);
        for (int i = 0; i < 3; i++) {
          float lo = te->m.emission[i] * ne.s;
          float Td = tri->m.diffuse[i] + tri->m.specular[i] * specd;
          Ld[i] = Td * lo;
        }
      } else {
        Ld[0] = Ld[1] = Ld[2] = 0.f;
      }
      vrec_t *vr = (rec && (max_bounces < 0 || n <= max_bounces)) ? &rec[n] : NULL;
      if (vr) {
        vr->tri = h.tri;
        for (int i = 0; i < 3; i++)
          vr->lo[i] = ne.ok ? sc->tris[ne.emitter].m.emission[i] * ne.s : 0.f;
        vr->specd = specd;
        vr->coeff = 0.f;
        vr->speci = 0.f;
      }
      n++;
      if (!(max_bounces >= 0 && k == max_bounces)) {
        float pr = xw_uniform(&st);
        if (pr < P_RR) {
          float psamp;
          v3 nd = sample_dir(tri, spec, tri->m.shininess, &psamp, &st);
          float speci = 0.f;
          if (tri->m.specular[0] != 0.f || tri->m.specular[1] != 0.f || tri->m.specular[2] != 0.f)
            speci = phong_coeff(&tri->m, nh, ray.d, nd);
          float coeff = (dot3(nd, nh) / psamp) / P_RR;
          for (int i = 0; i < 3; i++) {
            float Ti = tri->m.diffuse[i] / PI_F + tri->m.specular[i] * speci;
            M[i] = (M[i] * Ti) * coeff;
          }
          if (vr) { vr->coeff = coeff; vr->speci = speci; }
          ray.p = q;
          ray.d = nd;
          cont = 1;
        }
      }
    }
    for (int i = 0; i < 3; i++) L[i] = fmaf(Mp[i], Le[i] + Ld[i], L[i]);
    if (!cont) break;
    k++;
  }
  if (nrec) *nrec = n;
}

int oro_render_samples(void *p, int W, int H, int spp, int max_bounces, uint64_t seed,
                       int64_t s_begin, int64_t s_end, float *out, int64_t *casts) {
  oscene_t *sc = (oscene_t *)p;
  if (!sc || W <= 0 || H <= 0 || spp <= 0 || s_begin < 0 || s_end < s_begin ||
      s_end > (int64_t)W * H * spp) {
    set_err("bad render arguments");
    return -1;
  }
  int64_t total_casts = 0;
  int64_t n = s_end - s_begin;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : total_casts) num_threads(nthreads())
  for (int64_t i = 0; i < n; i++) {
    float L[3];
    int64_t cc = 0;
    trace_forward(sc, W, H, spp, max_bounces, seed, s_begin + i, L, &cc, NULL, NULL, NULL);
    out[3 * i] = L[0];
    out[3 * i + 1] = L[1];
    out[3 * i + 2] = L[2];
    total_casts += cc;
  }
  if (casts) *casts = total_casts;
  return 0;
}

/* toneMap, path_trace.cu:186-198 */
void oro_pixel_mean(const float *samples, int64_t npix, int spp, float *hdr, uint8_t *u8) {
  for (int64_t p = 0; p < npix; p++) {
    float tot[3] = {0.f, 0.f, 0.f};
    for (int s = 0; s < spp; s++)
      for (int i = 0; i < 3; i++) tot[i] += samples[(p * spp + s) * 3 + i] / (float)spp;
    for (int i = 0; i < 3; i++) {
      hdr[3 * p + i] = tot[i];
      if (u8) u8[3 * p + i] = (uint8_t)(255.f * tot[i] / (1 + tot[i]));
    }
  }
}

/* ------------------------------------------------------------------ */
/* inverse graph (inv_path_trace.cu:109-191, inv_scene.h:9-115)         */
/* ------------------------------------------------------------------ */
#define ACC_W 8
/* Edge::update, inv_scene.h:26-36 (DIFFUSE components; fp64 sums); acc NULL
 * = counting mode (oro_graph_casts: no bins) */
static void edge_update(double *acc, int nT, int dst, int src, float w, const float pix[3],
                        const float light[3], float f0) {
  if (!acc) return;
  double *e = acc + ((size_t)dst * nT + src) * ACC_W;
  float wf = w * f0;
  e[0] += (double)w;
  e[1] += (double)wf;
  for (int i = 0; i < 3; i++) {
    e[2 + i] += (double)(wf * pix[i]);
    e[5 + i] += (double)(wf * light[i]);
  }
}
static void trace_graph(const oscene_t *sc, int W, int H, int spp, int max_bounces,
                        uint64_t seed, int64_t gidx, const uint8_t *img, double *acc, int64_t *casts) {
  xorwow_t st;
  xw_init(&st, seed + (uint64_t)gidx);
  int64_t pix = gidx / spp;
  int r = (int)(pix / W), c = (int)(pix % W);
  ray_t ray = camera_ray(sc, &st, r, c, W, H);
  float weight = 1.f, f0 = 1.f;
  int dst = sc->nT;
  const uint8_t *px = img + ((size_t)r * W + c) * 3;
  float pixel[3] = {(float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f};
  const float zero[3] = {0.f, 0.f, 0.f};
  const double KW = ((1.0 / (double)INV_PI_F) / (double)P_RR) / (1.0 - 0.0);
  for (int k = 0;; k++) {
    hit_t h = intersect(sc, ray);
    if (casts) (*casts)++;
    if (h.tri < 0) break;
    const otri_t *tri = &sc->tris[h.tri];
    (void)xw_uniform(&st); /* isSpecular = u < P_SPEC (= 0): always false */
    int src = h.tri;
    edge_update(acc, sc->nT, dst, src, weight, pixel, zero, f0);
    v3 q = hit_point(ray, h.t);
    v3 nh = get_normal(tri, q);
    nee_t ne = nee_geometry(sc, tri, q, nh, weight, &st, casts);
    if (ne.ok) {
      float w2 = (float)ne.g;
      edge_update(acc, sc->nT, src, ne.emitter, w2, pixel, sc->tris[ne.emitter].m.emission,
                  INV_PI_F);
    }
    if (max_bounces >= 0 && k == max_bounces) break;
    float pr = xw_uniform(&st);
    if (pr >= P_RR) break;
    float psamp;
    v3 nd = sample_dir(tri, 0, 0.f, &psamp, &st);
    f0 = 1.f;
    weight *= dot3(nd, nh);
    weight = (float)((double)weight * KW);
    dst = src;
    ray.p = q;
    ray.d = nd;
  }
}

/* DataWrapper::compress, inv_scene.h:87-115 */
void oro_compress(int nT, const double *acc, float *data) {
  size_t sz = (size_t)(nT + 1) * nT;
  float *wts = data, *pix = data + sz, *lig = data + 4 * sz;
  float *ws = (float *)malloc(sizeof(float) * (size_t)(nT > 0 ? nT : 1));
  for (int dst = 0; dst <= nT; dst++) {
    float wt = 0.f;
    for (int src = 0; src < nT; src++) {
      const double *e = acc + ((size_t)dst * nT + src) * ACC_W;
      float w = logf((float)e[0] + 1);
      ws[src] = w;
      wt += w;
      float fs = (float)e[1];
      float wd = (fs != 0.f) ? fs : 1.f;
      for (int i = 0; i < 3; i++) {
        pix[((size_t)dst * nT + src) * 3 + i] = (float)e[2 + i] / wd;
        lig[((size_t)dst * nT + src) * 3 + i] = (float)e[5 + i] / wd;
      }
    }
    for (int src = 0; src < nT; src++) wts[(size_t)dst * nT + src] = (wt != 0.f) ? ws[src] / wt : 0.f;
  }
  free(ws);
}

/* Casts (path + shadow) of createGraph's integrator over rows [row_begin,
 * row_end): the C_bar of the graph roofline (bench.py).  The target image
 * only weights the bins, never the paths, so none is needed. */
int oro_graph_casts(void *p, int W, int H, int spp, int max_bounces, uint64_t seed, int row_begin, int row_end,
                    int64_t *casts) {
  oscene_t *sc = (oscene_t *)p;
  if (!sc || !casts || row_begin < 0 || row_end > H || row_begin > row_end) {
    set_err("bad graph arguments");
    return -1;
  }
  int nth = nthreads();
  uint8_t *img = (uint8_t *)calloc((size_t)W * H * 3, 1);
  if (!img) {
    set_err("out of memory");
    return -1;
  }
  int64_t b = (int64_t)row_begin * W * spp, e = (int64_t)row_end * W * spp, total = 0;
#pragma omp parallel num_threads(nth) reduction(+ : total)
  {
#ifdef _OPENMP
    int tid = omp_get_thread_num();
    int nt = omp_get_num_threads();
#else
    int tid = 0, nt = 1;
#endif
    int64_t chunk = (e - b + nt - 1) / nt;
    int64_t lo = b + chunk * tid, hi = lo + chunk < e ? lo + chunk : e;
    for (int64_t g = lo; g < hi; g++)
      trace_graph(sc, W, H, spp, max_bounces, seed, g, img, NULL, &total);  /* counting only */
  }
  *casts = total;
  free(img);
  return 0;
}

int oro_graph(void *p, int W, int H, int spp, int max_bounces, uint64_t seed, int row_begin,
              int row_end, const uint8_t *target, double *acc_out, float *data) {
  oscene_t *sc = (oscene_t *)p;
  if (!sc || row_begin < 0 || row_end > H || row_begin > row_end) {
    set_err("bad graph arguments");
    return -1;
  }
  size_t na = (size_t)(sc->nT + 1) * sc->nT * ACC_W;
  int nth = nthreads();
  double *accs = (double *)calloc(na * (size_t)nth, sizeof(double));
  if (!accs) {
    set_err("out of memory (per-thread graph bins)");
    return -1;
  }
  int64_t b = (int64_t)row_begin * W * spp, e = (int64_t)row_end * W * spp;
  int64_t n = e - b;
#pragma omp parallel num_threads(nth)
  {
#ifdef _OPENMP
    int tid = omp_get_thread_num();
    int nt = omp_get_num_threads();
#else
    int tid = 0, nt = 1;
#endif
    int64_t chunk = (n + nt - 1) / nt;
    int64_t lo = b + chunk * tid, hi = lo + chunk < e ? lo + chunk : e;
    for (int64_t g = lo; g < hi; g++)
      trace_graph(sc, W, H, spp, max_bounces, seed, g, target, accs + na * (size_t)tid, NULL);
  }
  double *acc = acc_out ? acc_out : (double *)malloc(na * sizeof(double));
  for (size_t i = 0; i < na; i++) {
    double s = 0.0;
    for (int t = 0; t < nth; t++) s += accs[na * (size_t)t + i];
    acc[i] = s;
  }
  if (data) oro_compress(sc->nT, acc, data);
  if (!acc_out) free(acc);
  free(accs);
  return 0;
}

/* ------------------------------------------------------------------ */
/* adjoint (new capability)                             */
/* ------------------------------------------------------------------ */
/* Per-thread record storage of the adjoint: max_bounces + 1 records, or for
 * unbounded paths (max_bounces < 0, the reference's own estimator) as many as
 * the path has -- counted by a first trace, then the same path traced again
 * with records (same seed, same draws). */
typedef struct {
  vrec_t *rec;
  float (*Mk)[3];
  int cap;
} adj_buf_t;
static void adj_buf_reserve(adj_buf_t *b, int n) {
  if (n <= b->cap) return;
  b->cap = n + 16;
  b->rec = (vrec_t *)realloc(b->rec, sizeof(vrec_t) * (size_t)b->cap);
  b->Mk = (float(*)[3])realloc(b->Mk, sizeof(float[3]) * (size_t)(b->cap + 1));
}
static void adjoint_sample(const oscene_t *sc, int W, int H, int spp, int max_bounces,
                           uint64_t seed, int64_t gidx, const float *adj, double *grad,
                           adj_buf_t *buf) {
  float L[3];
  int K = 0, esc = 0;
  if (max_bounces < 0) { /* unbounded: length first */
    trace_forward(sc, W, H, spp, max_bounces, seed, gidx, L, NULL, NULL, &K, &esc);
    adj_buf_reserve(buf, K);
  } else {
    adj_buf_reserve(buf, max_bounces + 1);
  }
  vrec_t *rec = buf->rec;
  trace_forward(sc, W, H, spp, max_bounces, seed, gidx, L, NULL, rec, &K, &esc);
  if (K == 0) return;
  int64_t pix = gidx / spp;
  float a[3];
  for (int i = 0; i < 3; i++) a[i] = adj[pix * 3 + i] / (float)spp;
  const float *Le = sc->tris[rec[0].tri].m.emission;
  float(*Mk)[3] = buf->Mk; /* prefix throughputs M_0..M_K */
  for (int i = 0; i < 3; i++) Mk[0][i] = 1.f;
  for (int k = 0; k < K; k++) {
    const omat_t *m = &sc->tris[rec[k].tri].m;
    for (int i = 0; i < 3; i++) {
      float Ti = m->diffuse[i] / PI_F + m->specular[i] * rec[k].speci;
      Mk[k + 1][i] = (Mk[k][i] * Ti) * rec[k].coeff;
    }
  }
  float S[3];
  for (int i = 0; i < 3; i++) {
    if (esc) {
      const omat_t *m = &sc->tris[rec[K - 1].tri].m;
      float Td = m->diffuse[i] + m->specular[i] * rec[K - 1].specd;
      S[i] = Le[i] + Td * rec[K - 1].lo[i];
    } else {
      S[i] = 0.f;
    }
  }
  for (int k = K - 1; k >= 0; k--) {
    const omat_t *m = &sc->tris[rec[k].tri].m;
    int continued = (k < K - 1) || esc;
    for (int i = 0; i < 3; i++) {
      float dLd = Mk[k][i];
      if (esc && k == K - 1) dLd = dLd + Mk[K][i];
      float g = dLd * rec[k].lo[i];
      if (continued) g = g + ((rec[k].coeff / PI_F) * Mk[k][i]) * S[i];
      grad[(size_t)rec[k].tri * 3 + i] += (double)(a[i] * g);
      float Td = m->diffuse[i] + m->specular[i] * rec[k].specd;
      float Gk = Le[i] + Td * rec[k].lo[i];
      float Ti = m->diffuse[i] / PI_F + m->specular[i] * rec[k].speci;
      S[i] = Gk + (Ti * rec[k].coeff) * S[i];
    }
  }
}

int oro_adjoint(void *p, int W, int H, int spp, int max_bounces, uint64_t seed, int row_begin,
                int row_end, const float *adj, double *grad) {
  oscene_t *sc = (oscene_t *)p;
  if (!sc || max_bounces > 62 || row_begin < 0 || row_end > H || row_begin > row_end) {
    set_err("bad adjoint arguments (max_bounces must be <= 62; < 0 = unbounded)");
    return -1;
  }
  size_t ng = (size_t)sc->nT * 3;
  int nth = nthreads();
  double *gs = (double *)calloc(ng * (size_t)nth, sizeof(double));
  int64_t b = (int64_t)row_begin * W * spp, e = (int64_t)row_end * W * spp;
  int64_t n = e - b;
#pragma omp parallel num_threads(nth)
  {
#ifdef _OPENMP
    int tid = omp_get_thread_num();
    int nt = omp_get_num_threads();
#else
    int tid = 0, nt = 1;
#endif
    adj_buf_t buf = {NULL, NULL, 0};
    int64_t chunk = (n + nt - 1) / nt;
    int64_t lo = b + chunk * tid, hi = lo + chunk < e ? lo + chunk : e;
    for (int64_t g = lo; g < hi; g++)
      adjoint_sample(sc, W, H, spp, max_bounces, seed, g, adj, gs + ng * (size_t)tid, &buf);
    free(buf.rec);
    free(buf.Mk);
  }
  for (size_t i = 0; i < ng; i++) {
    double s = 0.0;
    for (int t = 0; t < nth; t++) s += gs[ng * (size_t)t + i];
    grad[i] = s;
  }
  free(gs);
  return 0;
}
