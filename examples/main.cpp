// main.cpp — headless C++ counterpart of the reference front-end (src/main.rs:123-214),
// written against the C++ mirror API (include/ottomarcher.hpp) over libottomarcher.so.
//
// Same structure as main.rs: build the camera and random_scene, start the log thread that
// prints the samples_atom progress, deal pixels to num_cpus-1 render threads in 2730-pixel
// chunks, spawn them with render(&cam, &world, max_depth, tmin, tmax, spp, W, H, pixels_box,
// tid, &assigned, &atom).  Thread 0 drives the GPU for the whole frame; the others return.
// Instead of the SDL window (out of scope), every draw_to_sdl view (keys 0-6) is saved the
// way F12 saves the window (main.rs:473-476).
//
// --gpus N spreads the frame over devices 0..N-1 (MultiFrame: 8x8 tiles dealt round-robin,
// shards gathered over RCCL), still from render thread 0.
//
//   make -C examples && examples/ottomarcher_main [--width 1000] [--spp 200] [--fixed] [--gpus N] [--out DIR]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "ottomarcher.hpp"
#include "random_scene.hpp"

using namespace ottomarcher;

static void print_progress(double progress) {                                                 // main.rs:112-117
    const double p100 = std::round(100.0 * progress * 100.0) / 100.0;
    const double frac = std::fmod(p100, 1.0);
    std::fprintf(stderr, "%3llu.%02llu%%\r", (unsigned long long)(p100 - frac), (unsigned long long)(frac * 100.0));
}

int main(int argc, char** argv) {
    uint32_t image_width = 1000, samples_per_pixel = 200, max_depth = 50;                       // main.rs:126,145-146
    bool adaptive = true, torus = false;
    int gpus = 1;
    std::string out = "out";
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--width") image_width = (uint32_t)std::atoi(next());
        else if (a == "--spp") samples_per_pixel = (uint32_t)std::atoi(next());
        else if (a == "--max-depth") max_depth = (uint32_t)std::atoi(next());
        else if (a == "--fixed") adaptive = false;           // every pixel takes every sample (bench metric)
        else if (a == "--torus") torus = true;               // main.rs:73-81 block
        else if (a == "--out") out = next();
        else if (a == "--gpus") gpus = std::atoi(next());
        else { std::fprintf(stderr, "usage: %s [--width N] [--spp N] [--max-depth N] [--fixed] [--torus] [--gpus N] [--out DIR]\n", argv[0]); return 2; }
    }
    try {
        // IMAGE (main.rs:124-130)
        const float aspect_ratio = 3.0f / 2.0f;
        const float image_width_f = (float)image_width;
        const float image_height_f = image_width_f / aspect_ratio;
        const uint32_t image_height = (uint32_t)image_height_f;
        const uint32_t image_size = image_width * image_height;

        const Camera camera = default_camera(aspect_ratio);                                      // main.rs:132-143
        HittableList world = random_scene(0x5EED, torus);                                        // main.rs:147
        std::atomic<uint64_t> samples_atomic{0};                                                 // main.rs:148-149
        const FrozenHittableList frozen = world.freeze(camera);   // main.rs:198 (before the log thread: a throw
                                                                  // must not leave a joinable thread behind)
        std::unique_ptr<MultiFrame> multi;
        if (gpus > 1) {
            std::vector<int32_t> devices;
            for (int d = 0; d < gpus; ++d) devices.push_back(d);
            multi = std::make_unique<MultiFrame>(world, devices);
        }

        const uint64_t total_samples = (uint64_t)image_size * samples_per_pixel;
        std::atomic<bool> quit{false};
        std::thread log_thread([&]() {                                                           // main.rs:151-168
            const auto start = std::chrono::steady_clock::now();
            for (;;) {
                const uint64_t progress = samples_atomic.load(std::memory_order_relaxed);
                print_progress((double)progress / (double)total_samples);
                if (progress == total_samples || quit.load()) { print_progress((double)progress / (double)total_samples); break; }
                std::this_thread::sleep_for(std::chrono::milliseconds(500));
            }
            std::fprintf(stderr, "\n%.3f seconds\n",
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count());
        });

        const uint32_t hc = std::thread::hardware_concurrency();
        const uint32_t num_threads = hc > 1 ? hc - 1 : 1;                                        // main.rs:170
        const std::vector<uint32_t> assigned_thread = assign_threads(image_size, num_threads);  // main.rs:172-189
        std::vector<Pixel> pixels(image_size);                                                   // main.rs:192
        const PixelsBox pixels_box{&pixels};
        RenderOptions opt;
        opt.adaptive = adaptive;
        std::fprintf(stderr, "Running %u threads\n", num_threads);
        std::vector<std::thread> handlers;
        std::vector<std::string> errors(num_threads);
        for (uint32_t i = 0; i < num_threads; ++i) {                                             // main.rs:200-214
            handlers.emplace_back([&, i]() {
                try {
                    if (multi) {   // thread 0 drives every GPU; the others return, as in render()
                        if (i == 0)
                            multi->render(camera, max_depth, 0.001f, 100.0f, samples_per_pixel, image_width,
                                          image_height, pixels_box, samples_atomic, opt);
                    } else {
                        render(camera, frozen, max_depth, 0.001f, 100.0f, samples_per_pixel, image_width,
                               image_height, pixels_box, i, assigned_thread, samples_atomic, opt);
                    }
                } catch (const std::exception& e) {
                    errors[i] = e.what();
                }
            });
        }
        for (auto& h : handlers) h.join();
        quit = true;
        log_thread.join();
        for (const auto& e : errors)
            if (!e.empty()) { std::fprintf(stderr, "%s\n", e.c_str()); return 1; }

        // draw_to_sdl views (main.rs:360-437), saved like F12 (main.rs:473-476)
        static const char* names[7] = {"normal", "samples", "samples_blur", "depth", "depth_blur", "ids", "ids_blur"};
        std::filesystem::create_directories(out);
        for (int view = 0; view < 7; ++view) {
            const std::vector<uint8_t> rgb = display(frozen, pixels, image_width, image_height, view);
            const std::string path = out + "/" + names[view] + ".bmp";
            write_bmp(path, rgb, image_width, image_height);
            std::printf("wrote %s\n", path.c_str());
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
