// rs_internal.h — host <-> kernel launch interface (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rs_layout.h"

namespace rs {

constexpr int kBlock = 256;      // 4 waves of 64
constexpr int kStackMax = 32;    // per-thread BVH stack entries (LDS), host enforces tree depth

// One batch of camera samples: items = n_pix_local * n_samp_batch, item -> (sample, pixel).
struct PathParams {
    uint64_t n_items;
    uint32_t n_pix_local;   // pixels on the row lattice
    uint32_t width, height;
    uint32_t row_begin, row_step;
    uint32_t sqrt_spp;
    uint32_t s0;            // first sample index of the batch
    uint32_t depth;
    uint64_t key_base;      // splitmix64(splitmix64(seed) ^ pass)
    const uint8_t* mask;    // device, W*H or null
};

struct FinalParams {
    uint32_t n_pix_local, width, row_begin, row_step;
    uint32_t n_samples;
    int32_t gamma;
    const uint8_t* mask;
};

// Megakernel: one thread per (pixel, sample) path; radiance -> rad[c * n_items + item].
hipError_t launch_path_mega(const DScene& s, const DCamera& c, const PathParams& p, bool spheres_only, double* rad,
                            unsigned long long* seg_counters, hipStream_t st);
hipError_t launch_probe_hit(const DScene& s, const double* rays, uint32_t n, double tmin, double tmax, double* out,
                            hipStream_t st);
// acc[c * n_pix + pixel] += sum over the batch's samples in sample order (deterministic).
hipError_t launch_accumulate(const double* rad, double* acc, uint32_t n_pix, uint32_t n_samp_batch, int first_batch,
                             hipStream_t st);
// into_color + RGBA f32 store into the full frame.
hipError_t launch_finalize(const double* acc, float* out_rgba, const FinalParams& p, hipStream_t st);

}  // namespace rs
