/*
 * oracle/rtg_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference CPU raytracer (raytracer.h +
 * raytraceStack.h + algebra.h + vec.h + the commented-out per-pixel loop of
 * main.cpp:383-453).  It is the CHECKER for the HIP kernel: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product (librtg.so) never links or calls it.
 *
 * Pinning: bit-exact (NaN payloads included) against the reference itself
 * built from /root/reference by oracle/build_ref.sh (tests/test_oracle.py), and
 * against the committed golden fixtures in tests/golden/ that the reference
 * produced (tests/golden/make_golden.py).  Parity is therefore PINNED.
 *
 * The structure deliberately follows the reference literally (snapshot stack
 * with silent push-drop, the shared `colourSum` return register, double
 * islands) rather than the restructured form the GPU kernel uses, so that the
 * two are independent formulations.  Every function cites the reference line
 * it restates.  Arithmetic is written in the reference's exact operation order;
 * build with -O2 -ffp-contract=off and no fast-math (oracle/Makefile).
 *
 * Deviation from the reference (documented in DESIGN.md): the background
 * material's `opacity` is read uninitialised by the reference
 * (raytracer.h:694-697, main.cpp:423-426); here it is 0, which is what the
 * reference produces under the deterministic recipe of SURVEY.md §8c.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#include "rtg_oracle.h"

typedef struct { float x, y, z; } OVec;                     /* vec.h:27-29 */
typedef struct { OVec origin, dir, intensity; } ORay;       /* ray.h:9-14 */
typedef struct { OVec matte, gloss; float opacity, refr; } OMat; /* material.h:8-14 */
typedef struct { OVec pos; float radius; OMat mat; } OSph;  /* sphere.h:9-14 */
typedef struct { OVec pos, col; } OLight;                   /* raytracer.h:20-25 */
typedef struct { OSph object; OVec point, normal; float squaredDist; } OIsect; /* intersection.h:7-18 */

/* vec.h:31-41, expanded in exactly the macro's operation order. */
static inline OVec v3(float a, float b, float c) { OVec r = {a, b, c}; return r; }
static inline OVec vadd(OVec a, OVec b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline OVec vsub(OVec a, OVec b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline OVec vmul(OVec a, OVec b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline OVec vsmul(float k, OVec b) { return v3(k * b.x, k * b.y, k * b.z); }
static inline float vdot(OVec a, OVec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline OVec vnorm(OVec v) { float l = 1.f / sqrtf(vdot(v, v)); return vsmul(l, v); }

/* Per-thread counters (ray-sphere tests etc.). */
typedef struct { uint64_t sphere_tests, nodes, contain_tests; } OCount;

/* raytracer.h:81-141 */
static int raySphere(const OSph* s, const ORay* ray, float* t, OCount* cnt) {
  const float kEPSILON = 1.0e-5f;
  int result = 0;
  cnt->sphere_tests++;
  OVec d = vsub(ray->origin, s->pos);
  const float a = vdot(ray->dir, ray->dir);
  const float b = 2.0f * vdot(ray->dir, d);
  const float c = vdot(d, d) - (s->radius * s->radius);
  const float radicand = (b * b) - (4.0f * a * c);
  if (radicand >= 0.0) {
    const float root = sqrtf(radicand);
    const float denom = 2.0f * a;
    const float u[2] = {(-b + root) / denom, (-b - root) / denom};
    float smallestT = 10000.f;
    for (int i = 0; i < 2; ++i)
      if (u[i] > kEPSILON)
        if (u[i] < smallestT) { smallestT = u[i]; result = 1; }
    *t = smallestT;
  }
  return result;
}

/* raytracer.h:145-194 */
static int calcIntersection(const OSph* sph, unsigned n, const ORay* ray, OIsect* is,
                            OCount* cnt) {
  const float kMaxRenderDist = 1000.f;
  float minT = kMaxRenderDist;
  int found = 0;
  for (int i = 0; i < (int)n; ++i) {
    float t;
    if (raySphere(&sph[i], ray, &t, cnt)) {
      if (t < minT) {
        is->point = vadd(ray->origin, vsmul(t, ray->dir));
        is->normal = vnorm(vsub(is->point, sph[i].pos));
        OVec dist = vsmul(t, ray->dir);
        is->squaredDist = vdot(dist, dist);
        found = 1;
        is->object = sph[i];
        minT = t;
      }
    }
  }
  return found;
}

/* raytracer.h:235-241 */
static int isSignificant(OVec c) {
  const float k = 0.001f;
  return (c.x >= k) || (c.y >= k) || (c.z >= k);
}

/* raytracer.h:245-270 */
static int primaryContainer(const OSph* sph, unsigned n, OVec pt, OCount* cnt) {
  const float kEPSILON = 1.0e-6f;
  for (int i = 0; i < (int)n; ++i) {
    cnt->contain_tests++;
    const float r = sph[i].radius + kEPSILON;
    OVec dist = vsub(pt, sph[i].pos);
    if (vdot(dist, dist) <= (r * r)) return i;
  }
  return -1;
}

/* raytracer.h:272-309 */
static int hasClearLineOfSight(const OSph* sph, unsigned n, OVec A, OVec B, OCount* cnt) {
  OVec dir = vsub(B, A);
  const float gap = vdot(dir, dir);
  ORay ray;
  ray.dir = vnorm(dir);
  ray.origin = A;
  ray.intensity = v3(0.f, 0.f, 0.f); /* unused by calcIntersection */
  OIsect closest;
  if (calcIntersection(sph, n, &ray, &closest, cnt))
    if (closest.squaredDist < gap) return 0;
  return 1;
}

/* raytracer.h:313-367 */
static OVec calculateMatte(const OSph* sph, unsigned n, const OLight* lg, unsigned m,
                           const OIsect* is, OCount* cnt) {
  OVec sum = v3(0.f, 0.f, 0.f);
  for (int i = 0; i < (int)m; ++i) {
    const OLight L = lg[i];
    if (hasClearLineOfSight(sph, n, is->point, L.pos, cnt)) {
      OVec dist = vsub(L.pos, is->point);
      OVec dir = vnorm(dist);
      const float incidence = vdot(is->normal, dir);
      if (incidence > 0.f) {
        const float dm2 = vdot(dist, dist);
        const float intensity = incidence / dm2;
        sum = vadd(sum, vsmul(intensity, L.col));
      }
    }
  }
  return sum;
}

/* raytracer.h:370-403 — note the double-precision island.  cl: the OpenCL
 * kernel's all-float version, raytrace_kernel.cl:399-432. */
static float polarisedReflection(float n1, float n2, float cosA1, float cosA2, int cl) {
  const float kEPSILON = 1.0e-6f;
  const float left = n1 * cosA1;
  const float right = n2 * cosA2;
  if (cl) {
    const float numerator = left - right;
    float denominator = left + right;
    denominator *= denominator;
    if (denominator < kEPSILON) return 1.f;
    float reflection = (numerator * numerator) / denominator;
    if (reflection > 1.f) reflection = 1.f;
    return reflection;
  }
  double numerator = left - right;     /* float subtract, then widen */
  double denominator = left + right;   /* float add, then widen */
  denominator *= denominator;
  if (denominator < kEPSILON) return 1.f;
  float reflection = (float)((numerator * numerator) / denominator);
  if (reflection > 1.f) reflection = 1.f;
  return reflection;
}

/* algebra.h:10-14 */
static int isZero(float x) { return fabsf(x) < 0.001f; }

/* algebra.h:22-65 */
static int solveQuadratic(float a, float b, float c, float* roots) {
  if (isZero(a)) {
    if (isZero(b)) return 0;
    roots[0] = -c / b;
    return 1;
  }
  const float radicand = (b * b) - (4.f * a * c);
  if (isZero(radicand)) {
    roots[0] = -b / (2.f * a);
    return 1;
  }
  const float root = sqrtf(radicand);
  const float denom = 2.0f * a;
  roots[0] = (-b + root) / denom;
  roots[1] = (-b - root) / denom;
  return 2;
}

static OMat bgMaterial(void) {
  /* raytracer.h:694-697 / main.cpp:423-426: setMatteGlossBalance(0, black,
   * black) gives matte = (float)(1.0-0.0)*0 = 0, gloss = 0*0 = 0; n = 1.00f;
   * opacity uninitialised in the reference -> 0 (see header). */
  OMat m;
  memset(&m, 0, sizeof m);
  m.refr = 1.00f;
  return m;
}

/* raytracer.h:642-815 */
static ORay calculateRefraction(const OSph* sph, unsigned n, const OIsect* is, ORay inc,
                                const OMat* refrMat, OMat* tgt, float* outR, OCount* cnt,
                                int cl) {
  float cosA1 = vdot(inc.dir, is->normal);
  float sinA1 = 0.f;
  if (cosA1 <= -1.0) { cosA1 = -1.f; sinA1 = 0.f; }
  else if (cosA1 >= +1.f) { cosA1 = 1.f; sinA1 = 0.f; }
  /* :683, f64 sqrt (1.0 is a double literal); raytrace_kernel.cl:507 has the
   * same expression, and an OpenCL device with fp64 (gfx950) evaluates it in
   * double too, so both modes share it (pinned: tests/test_gpu_parity.py
   * test_opencl_reference_kernel_pins_oracle). */
  else { sinA1 = (float)sqrt(1.0 - (double)(cosA1 * cosA1)); }

  const float kSmallShift = 0.01f;
  {
    OVec testPt = vadd(vsmul(kSmallShift, inc.dir), is->point);  /* :690-691 */
    int container = primaryContainer(sph, n, testPt, cnt);
    if (container != -1) *tgt = sph[container].mat;
    else *tgt = bgMaterial();
  }
  const float ratio = refrMat->refr / tgt->refr;                  /* :712-714 */
  const float sinA2 = ratio * sinA1;                              /* :718 */
  if (sinA2 <= -1.f || sinA2 >= 1.f) { *outR = 1.f; }             /* :721-730 dead store */

  float roots[2];
  const int ns = solveQuadratic(1.f, (2.f * cosA1), (1.f - (1.f / (ratio * ratio))), roots);
  float maxAlignment = (float)-0.1;                               /* :750 */
  OVec dir = v3(0.f, 0.f, 0.f);
  for (int i = 0; i < ns; ++i) {
    OVec cur = vadd(inc.dir, vsmul(roots[i], is->normal));        /* :759-760 */
    float alignment = vdot(inc.dir, cur);
    if (alignment > maxAlignment) { maxAlignment = alignment; dir = cur; }
  }
  float cosA2 = sqrtf(1.f - (sinA2 * sinA2));                     /* :776, f32 sqrt */
  if (cosA1 < 0.f) cosA2 = -cosA2;
  const float Rs = polarisedReflection(refrMat->refr, tgt->refr, cosA1, cosA2, cl);
  const float Rp = polarisedReflection(refrMat->refr, tgt->refr, cosA2, cosA1, cl);
  *outR = (float)((double)(Rs + Rp) * 0.5);                       /* :798 (exact either way) */

  ORay out;
  out.intensity = vsmul((1.f - *outR), inc.intensity);            /* :807 */
  out.origin = is->point;
  out.dir = dir;
  return out;
}

/* raytracer.h:817-842 */
static ORay calculateReflection(const OIsect* is, ORay inc) {
  const float perp = 2.f * vdot(inc.dir, is->normal);
  OVec rd = vnorm(vsub(inc.dir, vsmul(perp, is->normal)));
  ORay out;
  out.dir = rd;
  out.intensity = inc.intensity;
  out.origin = vadd(is->point, vsmul(0.01f, rd));
  return out;
}

/* raytraceStack.h:13-68 */
typedef struct {
  ORay ray;
  int traceDepth, stage;
  OVec colour;
  OIsect isect;
  OMat refrMat;
  float R;
} OSnap;
#define ORACLE_MAX_STACK 64
typedef struct { OSnap el[ORACLE_MAX_STACK]; int top, maxSize; } OStack;
static void stInit(OStack* s, int S) { s->top = -1; s->maxSize = S; }
static int stEmpty(const OStack* s) { return s->top < 0; }
static void stPush(OStack* s, const OSnap* e) {
  if (!(s->top >= s->maxSize - 1)) s->el[++s->top] = *e;  /* silent drop when full */
}

/* raytracer.h:410-636 */
static OVec rayTrace(const OSph* sph, unsigned n, const OLight* lg, unsigned m, ORay ray,
                     OMat refrMat, int traceDepth, int S, OCount* cnt, int cl) {
  const int kMaxTraceDepth = 0x7FFFFFFF - 1;  /* RSIZE_MAX - 1 (Win32 value) */
  OVec colourSum = v3(0.f, 0.f, 0.f);
  OStack st;
  stInit(&st, S);
  OSnap cur;
  memset(&cur, 0, sizeof cur);
  cur.ray = ray;
  cur.traceDepth = traceDepth;
  cur.stage = 0;
  cur.colour = colourSum;
  cur.refrMat = refrMat;
  stPush(&st, &cur);
  while (!stEmpty(&st)) {
    cur = st.el[st.top];
    st.top--;
    switch (cur.stage) {
      case 0: {
        cnt->nodes++;
        if (calcIntersection(sph, n, &cur.ray, &cur.isect, cnt)) {
          if (cur.traceDepth <= kMaxTraceDepth) {
            if (isSignificant(cur.ray.intensity)) {
              const float opacity = cur.isect.object.mat.opacity;
              const float transparency = 1.f - opacity;
              if (opacity > 0.f) {
                OVec t = vmul(cur.ray.intensity, cur.isect.object.mat.matte);
                t = vsmul(opacity, t);
                OVec mc = calculateMatte(sph, n, lg, m, &cur.isect, cnt);
                t = vmul(mc, t);
                cur.colour = vadd(t, cur.colour);
              }
              float R = 0.f;
              if (transparency > 0.f) {
                ORay rr;
                rr.dir = cur.ray.dir;
                rr.intensity = vsmul(transparency, cur.ray.intensity);
                rr.origin = cur.ray.origin;
                OMat tgt;
                ORay refracted = calculateRefraction(sph, n, &cur.isect, rr, &cur.refrMat,
                                                     &tgt, &R, cnt, cl);
                cur.R = R;
                cur.stage = 1;
                stPush(&st, &cur);
                OSnap ns;
                memset(&ns, 0, sizeof ns);
                ns.ray = refracted;
                ns.traceDepth = traceDepth + 1;  /* the parameter, :527 */
                ns.stage = 0;
                ns.colour = v3(0.f, 0.f, 0.f);
                ns.refrMat = tgt;
                stPush(&st, &ns);
              }
              colourSum = cur.colour;
            }
          }
        } else {
          colourSum = vmul(cur.ray.intensity, cur.refrMat.matte);  /* :544 */
        }
        break;
      }
      case 1: {
        cur.colour = vadd(colourSum, cur.colour);                    /* :553 */
        OVec rc = v3(1.f, 1.f, 1.f);
        float transparency = 1.f - cur.isect.object.mat.opacity;
        float prod = transparency * cur.R;
        rc = vsmul(prod, rc);
        OVec g = vsmul(cur.refrMat.opacity, cur.isect.object.mat.gloss);
        rc = vadd(rc, g);
        rc = vmul(cur.ray.intensity, rc);
        if (isSignificant(rc)) {
          ORay rr;
          rr.dir = cur.ray.dir;
          rr.intensity = rc;
          rr.origin = cur.ray.origin;
          ORay reflected = calculateReflection(&cur.isect, rr);
          cur.stage = 2;
          stPush(&st, &cur);
          OSnap ns;
          memset(&ns, 0, sizeof ns);
          ns.ray = reflected;
          ns.traceDepth = traceDepth + 1;  /* :605 */
          ns.stage = 0;
          ns.colour = v3(0.f, 0.f, 0.f);
          ns.refrMat = cur.refrMat;
          stPush(&st, &ns);
          /* raytrace_kernel.cl:835-845 reuses currSnapshot as the child (colour
           * 0) before `colourSum = currSnapshot.colour` */
          if (cl) { colourSum = ns.colour; break; }
        }
        colourSum = cur.colour;
        break;
      }
      case 2: {
        cur.colour = vadd(colourSum, cur.colour);                    /* :622 */
        colourSum = cur.colour;
        break;
      }
    }
  }
  return colourSum;
}

/* main.cpp:411-452 (commented-out CPU loop). */
static void shadePixel(const OSph* sph, unsigned n, const OLight* lg, unsigned m, unsigned W,
                       unsigned H, float zoom, float aa, int S, unsigned gid, float* dst,
                       OCount* cnt, int cl) {
  const float xs = 16.f / ((float)W);
  const float ys = 12.f / ((float)H);
  const float asp = 16.f / 12.f;
  const float st = xs / aa;
  const float tot = aa * aa;
  const float inv = 1.f / tot;
  const float pxX = ((((float)(gid % W) - (W * 0.5f))) * xs);
  const float pxY = ((H * 0.5f) - ((float)(gid / W))) * ys;
  ORay ray;
  ray.origin = v3(0.f, 0.f, 0.f);
  ray.intensity = v3(1.f, 1.f, 1.f);
  OVec pix = v3(0.f, 0.f, 0.f);
  OMat bg = bgMaterial();
  for (int i = 0; i < aa; ++i) {
    for (int j = 0; j < aa; ++j) {
      float x = (pxX + (float)(((float)j) * st)) * asp;
      float y = (pxY + (float)(((float)i) * st));
      ray.dir = vnorm(v3(x, y, zoom));
      OVec c = rayTrace(sph, n, lg, m, ray, bg, 0, S, cnt, cl);
      c = vsmul(inv, c);
      pix = vadd(pix, c);
    }
  }
  dst[0] = pix.x;
  dst[1] = pix.y;
  dst[2] = pix.z;
}

typedef struct {
  const OSph* sph; unsigned n; const OLight* lg; unsigned m;
  unsigned W, H; float zoom, aa; int S, cl;
  const unsigned* rows; unsigned nrows; float* out;
  volatile unsigned next; pthread_mutex_t mu;
  OCount total;
} Job;

static void* worker(void* p) {
  Job* j = (Job*)p;
  OCount c = {0, 0, 0};
  for (;;) {
    pthread_mutex_lock(&j->mu);
    unsigned k = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (k >= j->nrows) break;
    unsigned y = j->rows[k];
    for (unsigned x = 0; x < j->W; ++x)
      shadePixel(j->sph, j->n, j->lg, j->m, j->W, j->H, j->zoom, j->aa, j->S, y * j->W + x,
                 j->out + ((size_t)k * j->W + x) * 3, &c, j->cl);
  }
  pthread_mutex_lock(&j->mu);
  j->total.sphere_tests += c.sphere_tests;
  j->total.nodes += c.nodes;
  j->total.contain_tests += c.contain_tests;
  pthread_mutex_unlock(&j->mu);
  return 0;
}

static int render_rows(const void* spheres, unsigned n, const void* lights, unsigned m,
                       unsigned W, unsigned H, float zoom, float aliasFactor, int stackSize,
                       const unsigned* rows, unsigned nrows, float* out, int nthreads,
                       unsigned long long* counters, int cl) {
  if (stackSize < 1 || stackSize > ORACLE_MAX_STACK) return -1;
  Job j;
  memset(&j, 0, sizeof j);
  j.cl = cl;
  j.sph = (const OSph*)spheres; j.n = n; j.lg = (const OLight*)lights; j.m = m;
  j.W = W; j.H = H; j.zoom = zoom; j.aa = aliasFactor; j.S = stackSize;
  j.rows = rows; j.nrows = nrows; j.out = out;
  pthread_mutex_init(&j.mu, 0);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if (nthreads == 1) {
    worker(&j);
  } else {
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], 0, worker, &j);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
  }
  pthread_mutex_destroy(&j.mu);
  if (counters) {
    counters[0] = j.total.sphere_tests;
    counters[1] = j.total.nodes;
    counters[2] = j.total.contain_tests;
  }
  return 0;
}

int oracle_render_rows(const void* spheres, unsigned n, const void* lights, unsigned m,
                       unsigned W, unsigned H, float zoom, float aliasFactor, int stackSize,
                       const unsigned* rows, unsigned nrows, float* out, int nthreads,
                       unsigned long long* counters) {
  return render_rows(spheres, n, lights, m, W, H, zoom, aliasFactor, stackSize, rows, nrows,
                     out, nthreads, counters, 0);
}

/* The semantics of the reference's OpenCL kernel (raytrace_kernel.cl) under
 * IEEE arithmetic with correctly rounded division and square root: f32
 * Fresnel (:399-432), sinA1 in f64 as on the CPU path (:507, a double
 * literal), and the return register zeroed by the reflection push
 * (:835-845); the stack capacity is the caller's (5 in the .cl, :58).  Pinned
 * bit for bit against the .cl itself, compiled for gfx950 with
 * -cl-fp32-correctly-rounded-divide-sqrt -ffp-contract=off
 * (oracle/build_ref_cl.sh, tests/test_gpu_parity.py
 * test_opencl_reference_kernel_pins_oracle).  The author's own image of it,
 * testPPM.ppm, used OpenCL's relaxed division/sqrt and contraction and is not
 * reproducible bit for bit. */
int oracle_render_rows_cl(const void* spheres, unsigned n, const void* lights, unsigned m,
                          unsigned W, unsigned H, float zoom, float aliasFactor, int stackSize,
                          const unsigned* rows, unsigned nrows, float* out, int nthreads) {
  return render_rows(spheres, n, lights, m, W, H, zoom, aliasFactor, stackSize, rows, nrows,
                     out, nthreads, 0, 1);
}

/* algebra.h:68-91 */
float oracle_max_colour(const float* fb, unsigned long long npx) {
  float mx = 0.f;
  for (unsigned long long i = 0; i < npx * 3; ++i)
    if (fb[i] > mx) mx = fb[i];
  if (mx == 0.f) mx = 1.f;
  return mx;
}

/* main.cpp:43-91 savePPM pixel conversion: (unsigned char)(min(1,c)*255/max).
 * The float->unsigned char cast of an out-of-range value is UB in C++; the
 * reference's x86 build (MSVC/gcc/clang alike) truncates to a 32-bit int with
 * cvttss2si (INT_MIN for NaN / out of range) and keeps the low byte. */
static unsigned char ppm_byte(float c, float mx) {
  float m = (c < 1.f) ? c : 1.f;  /* std::min(1.f, c) */
  float v = m * 255 / mx;
  int32_t i;
  if (v > -2147483649.0f && v < 2147483648.0f) i = (int32_t)v;
  else i = INT32_MIN;
  return (unsigned char)(i & 0xFF);
}

void oracle_ppm_bytes(const float* fb, unsigned long long npx, float mx, unsigned char* out) {
  for (unsigned long long i = 0; i < npx * 3; ++i) out[i] = ppm_byte(fb[i], mx);
}
