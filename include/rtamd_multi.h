/*
 * rtamd_multi — Scene::renderScene over several GPUs of one node from ONE process, RCCL
 * over xGMI (librtamd_multi.so; links librtamd.so and librccl.so).
 *
 * Replaces, for `as2 --gpus N` (the drop-in CLI, main.cpp:40-85 + options.cpp:7-16):
 *
 *   reference                                          this ABI
 *   -------------------------------------------------  ------------------------------------
 *   renderScene's thread pool over 2000-pixel blocks   rows in row_block blocks interleaved
 *     (scene.cpp:13-48)                                  over the devices (rt_partition_row)
 *   output(r, c) = traceRay(...) into one RasterImage  each device renders its rows; RGB8
 *     (scene.cpp:31)                                     (and/or f64) rows sent to the first
 *                                                        device (ncclSend/ncclRecv, one group)
 *                                                        and de-interleaved there
 *   --intersection-only global max (scene.cpp:50-58)   ncclAllReduce(MAX) of the devices'
 *                                                        maxima, then each device normalises
 *
 * Every image equals the single-device render bit for bit: tested with partitions sharing
 * one GPU (device list with repeats: the same partition, normalisation and assembly code,
 * rows moved by device copies instead of RCCL; tests/test_gpu_parity.py) and, on a node
 * with >= 2 GPUs, over RCCL (skipped on one-GPU boxes).
 * The scene is uploaded to every device (a few MB).  Plain C ABI, as include/rtamd.h.
 */
#ifndef RTAMD_MULTI_H
#define RTAMD_MULTI_H
#include "rtamd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_multi rt_multi;

/* The builder's scene on `n_devices` HIP devices (devices[0] assembles the image) and one
 * RCCL communicator per device (ncclCommInitAll).  row_block <= 0 means 8.  A list that
 * repeats a device makes partitions sharing that GPU (no communicator: device copies). */
int rt_multi_create(const rt_builder* b, int n_devices, const int* devices, int row_block, rt_multi** out);
/* The same from a flat scene descriptor (include/rtamd.h). */
int rt_multi_create_desc(const rt_scene_desc* d, int n_devices, const int* devices, int row_block, rt_multi** out);
void rt_multi_destroy(rt_multi* m);

/* A whole image (p->row_begin 0, row_end height, row_step 1) into caller-owned host buffers,
 * either may be NULL: out_rgb (H*W*3 doubles, the RasterImage) and out_rgb8 (H*W*3 bytes,
 * writers.cpp:4-9).  counters: sums over the devices; progress: 0 then the total. */
int rt_multi_render(rt_multi* m, const rt_render_params* p, double* out_rgb, uint8_t* out_rgb8,
                    rt_progress_fn progress, void* user, rt_counters* counters);

/* Per-device render time of the last rt_multi_render (ms, wall clock of each device's
 * render call) and the gather + assembly time, for load-balance reports. */
int rt_multi_last_times(const rt_multi* m, double* render_ms /* n_devices */, double* gather_ms);

#ifdef __cplusplus
}
#endif
#endif /* RTAMD_MULTI_H */
