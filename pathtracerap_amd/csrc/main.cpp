// main.cpp -- command-line renderer (the reference's main.cpp:11-27):
// load a scene, allocate on the GPU, run the render loop, write Render.bmp.
//
//   pathtracer_amd <scene.txt> [out.bmp] [--res W H] [--iter N] [--bounces B] [--grid|--grid-fast|--bvh]
//                  [--pipelines P]
//
// Default: PT_ACCEL_GRID_FAST (the reference grid's image, bit for bit) with 16
// iterations in flight, each on its own HIP stream and hardware queue.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/pathtracer_amd.h"

int main(int argc, char** argv) {
    // one hardware queue per pipeline stream; read once when the HIP runtime starts
    // (the library sets the same default when it loads; an explicit choice wins)
    setenv("GPU_MAX_HW_QUEUES", "16", /*overwrite=*/0);
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s scene.txt [out.bmp] [--res W H] [--iter N] [--bounces B] "
                             "[--grid|--grid-fast|--bvh] [--pipelines P]\n", argv[0]);
        return 2;
    }
    pt_render_config cfg;
    pt_default_config(&cfg);
    pt_scene* s = pt_scene_create();
    if (pt_scene_load_config(s, argv[1]) < 0) { std::fprintf(stderr, "%s\n", pt_last_error()); return 1; }
    pt_scene_apply_settings(s, &cfg);
    const char* out = "Render.bmp";
    for (int i = 2; i < argc; i++) {
        if (!std::strcmp(argv[i], "--res") && i + 2 < argc) { cfg.width = std::atoi(argv[++i]); cfg.height = std::atoi(argv[++i]); }
        else if (!std::strcmp(argv[i], "--iter") && i + 1 < argc) cfg.iterations = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--bounces") && i + 1 < argc) cfg.max_bounces = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--bvh")) cfg.accel = PT_ACCEL_BVH;
        else if (!std::strcmp(argv[i], "--grid-fast")) cfg.accel = PT_ACCEL_GRID_FAST;
        else if (!std::strcmp(argv[i], "--grid")) cfg.accel = PT_ACCEL_GRID;
        else if (!std::strcmp(argv[i], "--pipelines") && i + 1 < argc) cfg.pipelines = std::atoi(argv[++i]);
        else out = argv[i];
    }
    if (pt_scene_build(s, cfg.grid, cfg.accel != PT_ACCEL_GRID) < 0) { std::fprintf(stderr, "%s\n", pt_last_error()); return 1; }
    pt_renderer* r = pt_renderer_create(&cfg);
    if (!r || pt_renderer_allocate_on_gpu(r, s) < 0) { std::fprintf(stderr, "%s\n", pt_last_error()); return 1; }
    auto t0 = std::chrono::high_resolution_clock::now();
    if (pt_renderer_render_loop(r, 0, cfg.iterations) < 0 || pt_renderer_synchronize(r) < 0) {
        std::fprintf(stderr, "%s\n", pt_last_error());
        return 1;
    }
    auto t1 = std::chrono::high_resolution_clock::now();
    double us = std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    long long seg = pt_renderer_segments(r);
    std::printf("Full run: %.0f microseconds, %lld ray segments, %.2f Mrays/s\n", us, seg, seg / us);
    if (pt_renderer_render_image(r, out, cfg.iterations) < 0) { std::fprintf(stderr, "%s\n", pt_last_error()); return 1; }
    pt_renderer_free(r);
    pt_scene_destroy(s);
    return 0;
}
