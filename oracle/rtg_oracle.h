/* oracle/rtg_oracle.h — TEST INFRASTRUCTURE ONLY (see rtg_oracle.c). */
#ifndef RTG_ORACLE_H
#define RTG_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* Render rows[0..nrows) of a W x H frame with the reference CPU algorithm
 * (raytracer.h) at stack capacity `stackSize` (RTSTACK_MAXSIZE = depth + 1).
 * spheres: 48-B reference `struct Sphere` records; lights: 24-B `struct Light`.
 * out: nrows*W*3 floats.  counters (optional, 3 entries): raySphere calls,
 * stage-0 snapshots processed, primaryContainer sphere checks. */
int oracle_render_rows(const void* spheres, unsigned n, const void* lights, unsigned m,
                       unsigned W, unsigned H, float zoom, float aliasFactor, int stackSize,
                       const unsigned* rows, unsigned nrows, float* out, int nthreads,
                       unsigned long long* counters);

/* Same, with the OpenCL kernel's semantics (raytrace_kernel.cl; see the .c). */
int oracle_render_rows_cl(const void* spheres, unsigned n, const void* lights, unsigned m,
                          unsigned W, unsigned H, float zoom, float aliasFactor, int stackSize,
                          const unsigned* rows, unsigned nrows, float* out, int nthreads);

/* algebra.h:68-91 maxColourValuePixelBuffer. */
float oracle_max_colour(const float* fb, unsigned long long npx);

/* main.cpp:66-81 byte conversion of savePPM (npx*3 bytes). */
void oracle_ppm_bytes(const float* fb, unsigned long long npx, float mx, unsigned char* out);

#ifdef __cplusplus
}
#endif
#endif
