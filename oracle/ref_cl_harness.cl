// oracle/ref_cl_harness.cl — TEST INFRASTRUCTURE: a harness around the
// reference's own OpenCL kernel, raytrace_kernel.cl (included in place from
// /root/reference/raytracer_gamma by oracle/build_ref_cl.sh; nothing of it is
// copied into the repo).  It pins the OpenCL-semantics oracle
// (oracle_render_rows_cl, oracle/rtg_oracle.c) and the kernel's kCL mode bit
// for bit.
//
// The reference kernel takes its sphere and light tables as two dynamically
// sized __local pointer arguments (raytrace_kernel.cl:880-881), whose LDS
// offsets an OpenCL runtime assigns at clSetKernelArg time
// (main.cpp:325-336).  This wrapper passes two fixed __local arrays instead,
// so a plain HIP module launch (hipModuleLaunchKernel, tests/clref.py) can run
// it: the reference copies sphere k and light k with work-item k of the group
// (raytrace_kernel.cl:890-907), so it needs sphNum, lgtNum <= the work-group
// size (64 here), as the reference's own host does (main.cpp:316-336).
// Every work-item writes dst[get_global_id(0)] (raytrace_kernel.cl:972) with
// no bounds check: the caller pads dst to the launched grid.
#include "raytrace_kernel.cl"

#define RTG_CL_MAX_SPHERES 64
#define RTG_CL_MAX_LIGHTS 64

__kernel __attribute__((reqd_work_group_size(64, 1, 1)))
void rtg_ref_cl_raytrace(__global struct Sphere* spheres, const unsigned int sphNum,
                         __global struct Light* lights, const unsigned int lgtNum,
                         const unsigned int kWidth, const unsigned int kHeight,
                         const float kZoom, const float kAliasFactor, __global Vec* dst) {
  __local struct Sphere lSpheres[RTG_CL_MAX_SPHERES];
  __local struct Light lLights[RTG_CL_MAX_LIGHTS];
  raytrace(spheres, sphNum, lights, lgtNum, kWidth, kHeight, kZoom, kAliasFactor, dst,
           lSpheres, lLights);
}
