// renderer.h -- MI355X wavefront renderer (Renderer.h:46-55 mirror).
//
// allocateOnGPU / renderLoop / renderImage / free keep the reference's
// entry points; underneath, each bounce is a persistent trace kernel
// (grid_fast / bvh; grid_fast after a counting sort of the live rays) and a
// shading kernel (BSDF scatter + block-local stable compaction + framebuffer
// accumulate of terminated rays), then a one-workgroup block-offset scan --
// no host round trip inside an iteration.  `pipelines` iterations run at once
// on their own HIP streams; their contributions merge in iteration order.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "scene.h"

namespace pt {

struct RenderConfig {            // Config.h + generateRaysKernel constants, at runtime
    int width = 1000, height = 800;       // RESOLUTION_X/Y
    int iterations = 500;                 // ITER
    int max_bounces = 5;                  // Renderer.cpp:550
    int accel = ACCEL_GRID_FAST;          // the reference grid's results, bit for bit, through the BLAS
    int grid[3] = {25, 25, 25};           // GRID_X/Y/Z
    int tail_drop = 0;                    // replicate ceil(n/32) launch truncation (Renderer.cpp:573)
    int block = 64;                       // bounce-kernel workgroup size = compaction chunk (64/128/256)
    int ray_sort = -1;                    // -1 auto (grid_fast: key 7), 0 off, 1..8 key layout (k_sort_hist)
    int pipelines = 16;                   // iterations in flight on their own HIP streams (1..kMaxPipes)
    double cam[3] = {0.0, 0.0, 920.0};    // Renderer.cpp:528
    double plane_z = 900.0;               // Renderer.cpp:543
    double plane_x0 = -10.0, plane_y0 = -4.0, plane_w = 20.0, plane_h = 16.0;  // Renderer.cpp:538-542
};

// Everything a kernel needs, passed by value as the kernel argument.
struct KParams {
    // scene (read-only, stays L2/MALL resident)
    const ModelRec* models;
    const ModelShade* shade;    // per model: material (shading pass)
    int nmodels;
    int gdim[3];
    const float4* tri_geom;     // 3 float4 per triangle: v0, e1, e2
    const float4* tri_normal;   // 1 float4 per triangle
    const int2* voxels;         // (start, end)
    const int* per_voxel;
    const Bvh4Node* bvh4;       // the BLAS, 4-wide: every BLAS path walks it (nullptr when the scene has none)
    const float4* bvh_tri_geom; // leaf-ordered triangle records, v0.w = triangle index
    int top_root[2], top_n[2];  // PT_LDS_TOP builds: the two largest meshes' 4-wide roots, nodes staged (<= kLdsTop)
    int* spill;                 // traversal-stack spill beyond the LDS entries, lane-minor
    int spill_stride;           // lanes in the spill layout
    // frame
    int width, height, npix, max_bounces, nblocks, chunk;
    float step_x, step_y, cam_x, cam_y, cam_z, plane_z;
    double plane_x0, plane_y0;
    float4* ray[2][3];          // ping-pong SoA planes: (o, pixel) (d, bounces) (color, -)
    float4* cache_hit;          // primary hit: dist, normal
    int* cache_model;
    float* image;               // W*H*3 accumulator (Pixel::color)
    int* blk_cnt;
    int* blk_off;
    int* dst_start;
    int* n_live;                // live rays per bounce
    unsigned long long* segments;      // [0] total, [1 + b] live rays entering bounce b, [65] diagnostics
    int debug;                          // timing-only ablation switches (PT_DEBUG_ABLATE); 0 in production
    int4* hs_pool;                      // ACCEL_GRID_FAST overflow hit sets (64-member blocks)
    int* hs_pool_next;                  // bump allocator, reset by k_scan every bounce
    int hs_pool_blocks;
    float4* hit4;                       // split trace/shade (ACCEL_BVH): per-slot dist, normal
    int* hitm;                          // per-slot model
    int* trace_next;                    // persistent trace: next unclaimed source block, reset by k_scan
    int trace_refill;                   // refill a wave's idle lanes once this many are idle
    int trace_rpl;                      // main trace launch: waves beyond ceil(n / (64 * trace_rpl)) exit at once (0: off)
    int trace_min_blocks;               // ... but at least this many waves run
    int trace_flags;                    // k_trace_bvh variant: 11 LDS model records, 10 global
    int* defer_slots;                   // k_trace_gf: slots whose hit set overflowed LDS (k_trace_deferred)
    int* defer_count;                   // reset by k_scan
    float* contrib;                     // pipelines > 1: this pipeline's per-iteration contributions (k_merge)
    int2* order;                        // ray sort: claim position -> (dense slot, source index); null: claim order
    int* sort_bins;                     // [kSortBins] rays per key, [kSortBins] scatter cursors; zeroed by k_scan
    unsigned short* sort_key;           // per source index of the previous bounce's pool
    int sort_mode;                      // key layout (k_sort_hist); 0 = no sort
    float sort_lo[3], sort_sc[3];       // origin cell = (o - lo) * sc, scene world box
    int* iter_dev;                      // hipGraph replay: k_bounce's iteration id (its `iter` argument is -1)
    int* cont;                          // drain continuations: rays a persistent trace handed on (SoA, stride cont_cap)
    int cont_cap;
    int* cont_count;                    // [level] records written by that launch, [kDrainLevels + level]
                                        // walk hand-ons it wrote (k_trace_gf; reset by k_scan)
    int cont_wcap;                      // walk hand-on records per launch (at the top of the buffer; 0: off)
    int* cont_next;                     // [level] of them claimed by the next tail launch (reset by k_scan)
    int drain_levels;                   // tail launches after the main one (PT_DRAIN_LEVELS); the last one
                                        // hands nothing on.  Record buffers alternate between levels
    int drain_dump;                     // hand a wave's rays on once the pool is exhausted and <= this many
                                        // lanes still trace (0: off; PT_DRAIN_DUMP overrides)
    int drain_dump_tail;                // the same for a tail launch that hands on again (PT_DRAIN_DUMP_TAIL)
    int tail_rpl;                       // tail launches: waves beyond ceil(records / (64 * tail_rpl)) exit at
                                        // once, so each lane resumes about tail_rpl records (PT_TAIL_RPL; 1 =
                                        // one wave per 64 records)
    int tail_refill;                    // a tail wave claims more records once this many lanes are idle
    int allphase_lanes;                 // k_trace_gf: every step kind each iteration once the rays are claimed
                                        // and at most this many lanes trace (PT_ALLPHASE_LANES; 0 = off)
    int defer_launch;                   // 0: k_trace_deferred is not launched (PT_DEFER_LAUNCH=0, timing
                                        // experiments); k_scan then counts a trace fault if any ray was deferred
    unsigned trace_iter_cap;            // persistent traces give up after this many loop iterations (a fault,
                                        // counted in segments[kTraceFaultCounter]); PT_TRACE_ITER_CAP overrides
};

constexpr int kMaxBounceCounters = 64;
constexpr int kDrainLevels = 4;          // most tail launches per trace (drain continuations)
constexpr int kDiagCounters = 96;        // diagnostic counters after the per-bounce ones (PT_TRACE_STATS builds)
// segments[] slot counting persistent-trace waves that hit trace_iter_cap and left
// rays untraced (their hit records are stale): any non-zero value invalidates the image
constexpr int kTraceFaultCounter = 7 + kMaxBounceCounters;
// segments[] slot counting rays k_trace_deferred traced (grid_fast hit sets that
// outgrew the overflow pool, or walks past the hand-on records' room); every build
constexpr int kDeferredRayCounter = 50 + kMaxBounceCounters;

struct KernelStats {
    double bounce_ms = 0, scan_ms = 0, primary_ms = 0, first_ms = 0, trace_ms = 0;
    double sort_ms = 0;                  // ray sort before each persistent trace (k_sort_hist/prefix/scatter)
    long long sort_launches = 0;
    long long bounce_launches = 0, scan_launches = 0, first_launches = 0;   // bounce_* = secondary bounces
    long long trace_launches = 0;        // k_trace_bvh (split trace/shade); bounce_* is then the shading pass
};

class Renderer {
public:
    explicit Renderer(const RenderConfig& cfg);
    ~Renderer();
    int allocateOnGPU(const Scene& scene);          // Renderer.cpp:65-130
    int clearImage();                                // initImageKernel (Renderer.cpp:557-565)
    int renderLoop(int first_iter, int n_iters);     // Renderer.cpp:567-648 (asynchronous)
    int renderImage(const std::string& path, int iterations_total);  // Renderer.cpp:15-63
    int readImage(float* host_rgb);
    int synchronize();
    void free();                                     // Renderer.cpp:132-148

    int setStream(hipStream_t s);
    int bindImage(float* device_rgb);
    int setProfiling(int on);              // 0 off, 1 every kernel group, 2 pipeline 0's trace phases
    int kernelStats(KernelStats* out);
    long long segments();
    long long traceFaults();                         // waves that gave up (see kTraceFaultCounter); -1 on error
    int pipelines() const { return npipes; }
    int segmentsPerBounce(long long* out, int n);
    int primaryHits(float* dist, float* normal, int* model);
    int intersectRays(int n, const float* orig, const float* dir, float* dist, float* normal, int* model);
    // test hook (grid_fast): walk certificates vs the exact walk on the same hit sets; 4 ints per ray
    int certifyCheck(int n, const float* orig, const float* dir, int* out4);

    RenderConfig cfg;
    std::string last_error;

private:
    int launchPrimary();
    void launchTrace(const KParams& k, hipStream_t st, int b);
    void launchBounce(const KParams& k, hipStream_t st, bool first, dim3 grid, int iter, int b, int accel);
    int allocPipe(KParams& k, size_t cap, hipStream_t st);
    int fail(hipError_t e, const char* what);
    void freeBuffers();
    int enqueueIteration(int q, hipStream_t st, int iter, int passes);
    void dropGraphs();
    int joinPipes(int np);
    int checkFaults();

    KParams kp{};                    // pipeline 0 (and everything the pipelines share)
    hipStream_t stream = nullptr;    // the caller's stream; pipeline 0 runs on it
    static constexpr int kMaxPipes = 32;
    int npipes = 1;
    KParams pk[kMaxPipes]{};         // pipeline i's parameters (pk[0] == kp)
    hipStream_t pstream[kMaxPipes]{};    // pstream[0] == stream; 1.. created here
    hipEvent_t merge_ev[kMaxPipes]{};    // last k_merge recorded on each pipeline
    hipEvent_t fork_ev = nullptr;
    hipGraphExec_t gexec[kMaxPipes]{};   // PT_GRAPH: pipeline i's bounce loop captured once, replayed per iteration
    bool use_graph = false;
    bool own_stream = false;
    bool stream_set = false;
    bool allocated = false;
    bool cache_valid = false;        // is_first_intersection_cached (Renderer.cpp:580)
    bool external_image = false;
    float* ext_image = nullptr;
    int profiling = 0;
    std::vector<void*> allocs;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> bounce_events, first_events, scan_events, trace_events, sort_events;
    bool split_trace = false;        // persistent k_trace_bvh / k_trace_gf + shading pass
    int trace_blocks = 0;
    int tail_blocks = 0;             // grid of k_trace_gf's tail launches (PT_TAIL_BLOCKS; default trace_blocks)
    int gf_flags = 9;                // k_trace_gf variant: 1 LDS model records, 8 phase scheduling
    bool gf_wide_lds = false;        // k_trace_gf default variants with 9..12 models: 12 LDS records (F | 32)
    bool bvh_wide_lds = false;       // k_trace_bvh default variant with 9..12 models: 12 LDS records (F = 43)
    KernelStats stats;
};

// Device math conformance hook (pt_selftest_math).
int selftest_math(int n, const float* x, const float* y, float* out, std::string* err);

}  // namespace pt
