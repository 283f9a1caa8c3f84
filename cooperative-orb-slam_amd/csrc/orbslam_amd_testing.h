/*
 * orbslam_amd_testing.h -- test and measurement hooks of liborbamd.so. Internal: not part of the
 * drop-in ABI (include/orbslam_amd.h). The tests and bench.py bind them through ctypes
 * (orbamd/_lib.py); no reference member maps to them and the product never calls them.
 */
#ifndef ORBSLAM_AMD_TESTING_H
#define ORBSLAM_AMD_TESTING_H
#include "../../include/orbslam_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test hook: the stages in `mask` (bit k of {pyramid, fast_cells, octree, blur, describe}) are not
 * launched by subsequent batched extractions of this handle (0 = every stage runs, the default). A
 * skipped stage leaves its buffers as the previous call left them; the tests use it to prove that
 * the bench's self-check detects a stage that stopped launching. Bit 3 (blur) only acts on frames that
 * take the separate blur (level-0 rows not 4-byte aligned); frames with aligned rows blur inside
 * describe (k_describe_blur), so for them skipping the blur means skipping describe (bit 4), and a
 * test that skips bit 3 alone on such frames must expect every output to stay correct. Skipping the
 * octree (bit 2) also skips the host path's pyramid copy that rides on its launch, so
 * orbx_host_pyramid_level reports no pyramid for that call. */
int orbx_debug_skip_stages(orbx_handle* h, int mask);

/* Measurement hook: on != 0 runs every stage of this handle's subsequent extractions in order on the
 * caller's stream (no side stream for the blur), so a kernel trace times each kernel alone; 0 = the
 * default fork/join schedule. Outputs are identical either way. */
int orbx_debug_serial(orbx_handle* h, int on);

/* Measurement hook (the L2-residency bound of DESIGN.md 6.0): on != 0 makes every frame of this
 * handle's subsequent batched extractions read frame 0's image and share one pyramid and one blurred
 * pyramid, so every stage reads data the launch keeps in L2; each frame's outputs are then frame 0's.
 * Never on in the product; 0 = off (the default). */
int orbx_debug_alias_frames(orbx_handle* h, int on);

/* Test hook: ORs `flag` (> 0) into the handle's sticky batch error word, as a failing device batch
 * would; the tests use it to show that host-path extractions (orbx_extract) neither clear nor hide it
 * and that orbx_check_error reports and clears it once. */
int orbx_debug_raise_error(orbx_handle* h, int flag, void* stream);

/* Test hook: one HIP runtime call that fails (hipEventElapsedTime over two never-recorded events) inside the
 * library's error handling; returns ORBX_EDEVICE, and the calling thread's HIP error state (hipGetLastError) must be
 * clean afterwards, so the failure does not resurface in the caller's next launch check. */
int orbx_debug_hip_failure(void);

/* Measurement query (host-only): 1 if a batched extraction of frames at `frames` (device pointer value, frame stride
 * and row pitch in bytes) blurs inside describe (k_describe_blur: level-0 rows 4-aligned), 0 if it takes the separate
 * blur (k_blur_strips + k_describe); bench.py prices describe's bytes by the form that ran. */
int orbx_describe_blur_fused(const void* frames, size_t frame_stride, size_t pitch);

/* Test hook: the device's restatement of glibc sinf/cosf (used by computeOrbDescriptor,
 * ORBextractor.cc:113) applied to n device floats; lets tests compare against host libm. */
int orbx_selftest_sincosf(const float* d_in, float* d_sin, float* d_cos, int n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ORBSLAM_AMD_TESTING_H */
