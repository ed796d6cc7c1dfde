// raytrace_main.cpp — the repository's `raytrace` program: the reference's main()
// (/root/reference/source.cpp:190-231) with render() (source.cpp:98-178) served by the GPU
// through include/ykgpu.h, plus the runtime render parameters BASELINE configs 2-5 need.
//
// This is NOT the reference's binary: its option parser and PNG writer are this file's own (the
// reference's are cxxopts and stb_image_write, which this repository does not vendor).  The
// reference's exact program — its cxxopts CLI, its stb PNG bytes — is the reference's own
// source.cpp with oracle/source_cpp_ykgpu.patch applied (tests/test_cli.py
// checks that build's PNG byte for byte against the reference's constexpr build).
//
// Kept from the reference: -h/--help, -v/--verbose, -o/--output, -l/--verbose-level and the
// positional output (source.cpp:197-216: help or no output → usage + exit 0; the last -l wins),
// the messages "rendering...", "rendering finished", "write to file : <f>", "success" / "error"
// with exit 1 (source.cpp:114,174-175,223-230), the default image (YK_IMAGE_WIDTH 400, YK_SPP 100,
// YK_MAX_DEPTH 50; source.cpp:43-53) and the reference scene (source.cpp:103-112), built with the
// same yk calls.  A bad argument is reported with a message and exit status 2 (the reference
// lets cxxopts' exception escape main and aborts).
//
// Added (render parameters are compile-time macros in the reference): --width, --spp,
// --depth, --scene, --scene-seed, --scene-file, --save-scene, --seed0, --precision, --rng,
// --device, --stats.  --seed0 fixes the per-sample seed base (seed0 + (y*W+x)*spp + s, the constexpr
// build's formula, source.cpp:154-158); without it every sample gets its own seed from a
// per-call std::random_device key (YK_SEED_RANDOM_DEVICE), like the reference's runtime build
// (source.cpp:159).  --precision fp32 renders render<float> (T = float, source.cpp:98);
// --rng xor128 seeds the reference's yk::xor128 (random.hpp:18-41) per sample instead of
// yk::mt19937.
// Verbose output: the reference's per-pixel / per-sample lines (levels 1-2) and, at level 3, every
// ray ray_color is called with (raytracer.hpp:21-25, from ykgpu_render_trace), in the
// reference's order, after the GPU render.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <random>
#include <string>
#include <vector>

#include "png_write.hpp"
#include "yk/scene.hpp"
#include "yk/ykgpu_bridge.hpp"

#ifndef YK_IMAGE_WIDTH
#define YK_IMAGE_WIDTH 400
#endif
#ifndef YK_SPP
#define YK_SPP 100
#endif
#ifndef YK_MAX_DEPTH
#define YK_MAX_DEPTH 50
#endif

namespace {

struct option_error {
  std::string what;
};

const char* kHelp =
    "raytracing program\n"
    "Usage:\n"
    "  raytrace [OPTION...] positional parameters\n"
    "\n"
    "  -h, --help                print usage\n"
    "  -v, --verbose             verbose output\n"
    "  -o, --output arg          filename of output\n"
    "  -l, --verbose-level arg   set verbose level\n"
    "      --width arg           image width (default: " "400" ")\n"
    "      --spp arg             samples per pixel (default: 100)\n"
    "      --depth arg           max bounce depth (default: 50)\n"
    "      --scene arg           ref4|lambert3|mixed12|walls2|rtiow5|final|glass (default: ref4)\n"
    "      --scene-seed arg      generator seed of final/glass (default: 42)\n"
    "      --scene-file arg      load the scene from a yk-scene file (overrides --scene)\n"
    "      --save-scene arg      write the scene to a yk-scene file\n"
    "      --seed0 arg           per-sample seed base (default: random_device)\n"
    "      --precision arg       fp64|fp32: the T of render<T> (default: fp64)\n"
    "      --rng arg             mt19937|xor128: the per-sample engine (default: mt19937)\n"
    "      --device arg          GPU index (default: 0)\n"
    "      --stats               print kernel time and throughput\n";

struct args {
  bool help = false, verbose_flag = false, stats = false;
  std::vector<uint32_t> levels;
  std::string output;
  bool have_output = false;
  uint32_t width = YK_IMAGE_WIDTH, spp = YK_SPP, depth = YK_MAX_DEPTH, scene_seed = 42;
  int device = 0;
  bool have_seed0 = false;
  uint32_t seed0 = 0;
  std::string precision = "fp64";
  std::string rng = "mt19937";
  std::string scene = "ref4";
  std::string scene_file, save_scene;
};

uint32_t to_u32(const std::string& opt, const std::string& v) {
  char* end = nullptr;
  const unsigned long long x = std::strtoull(v.c_str(), &end, 10);
  if (v.empty() || *end || x > 0xffffffffull || v[0] == '-')
    throw option_error{"Argument '" + v + "' failed to parse (option " + opt + ")"};
  return (uint32_t)x;
}

args parse(int argc, char** argv) {
  args a;
  int positional = 0;
  auto value = [&](int& i, const std::string& name, const std::string& inl) -> std::string {
    if (!inl.empty()) return inl;
    if (i + 1 >= argc) throw option_error{"Option '" + name + "' is missing an argument"};
    return argv[++i];
  };
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    std::string inl;
    if (s.rfind("--", 0) == 0 && s.size() > 2) {
      const size_t eq = s.find('=');
      if (eq != std::string::npos) {
        inl = s.substr(eq + 1);
        s = s.substr(0, eq);
      }
      const std::string n = s.substr(2);
      if (n == "help") a.help = true;
      else if (n == "verbose") a.verbose_flag = true;
      else if (n == "stats") a.stats = true;
      else if (n == "output") { a.output = value(i, n, inl); a.have_output = true; }
      else if (n == "verbose-level") {
        std::string v = value(i, n, inl);
        for (size_t p = 0; p <= v.size();) {  // cxxopts vector values: comma separated
          const size_t q = v.find(',', p);
          a.levels.push_back(to_u32(n, v.substr(p, q == std::string::npos ? std::string::npos : q - p)));
          if (q == std::string::npos) break;
          p = q + 1;
        }
      } else if (n == "width") a.width = to_u32(n, value(i, n, inl));
      else if (n == "spp") a.spp = to_u32(n, value(i, n, inl));
      else if (n == "depth") a.depth = to_u32(n, value(i, n, inl));
      else if (n == "scene-seed") a.scene_seed = to_u32(n, value(i, n, inl));
      else if (n == "device") a.device = (int)to_u32(n, value(i, n, inl));
      else if (n == "scene") a.scene = value(i, n, inl);
      else if (n == "scene-file") a.scene_file = value(i, n, inl);
      else if (n == "save-scene") a.save_scene = value(i, n, inl);
      else if (n == "seed0") { a.seed0 = to_u32(n, value(i, n, inl)); a.have_seed0 = true; }
      else if (n == "precision") a.precision = value(i, n, inl);
      else if (n == "rng") a.rng = value(i, n, inl);
      else throw option_error{"Option '" + n + "' does not exist"};
    } else if (s.size() > 1 && s[0] == '-') {
      for (size_t k = 1; k < s.size(); ++k) {
        const char c = s[k];
        const std::string rest = s.substr(k + 1);
        if (c == 'h') a.help = true;
        else if (c == 'v') a.verbose_flag = true;
        else if (c == 'o') { a.output = value(i, "o", rest); a.have_output = true; break; }
        else if (c == 'l') { a.levels.push_back(to_u32("l", value(i, "l", rest))); break; }
        else throw option_error{std::string("Option '") + c + "' does not exist"};
      }
    } else {
      // one positional argument, the output file (source.cpp:206)
      if (positional++ == 0) {
        a.output = s;
        a.have_output = true;
      } else {
        throw option_error{"unexpected second positional argument '" + s + "'"};
      }
    }
  }
  return a;
}

}  // namespace

int main(int argc, char* argv[]) {
  std::ios::sync_with_stdio(false);
  std::cout.tie(nullptr);

  args a;
  try {
    a = parse(argc, argv);
  } catch (const option_error& e) {
    std::cerr << "raytrace: " << e.what << " (see --help)" << std::endl;
    return 2;
  }
  if (a.help || !a.have_output) {
    std::cout << kHelp << std::endl;
    std::exit(EXIT_SUCCESS);
  }
  uint32_t verbose = 0;
  if (a.verbose_flag && !verbose) ++verbose;
  if (!a.levels.empty()) verbose = a.levels.back();

  const uint32_t W = a.width, H = yk_image_height_for(W);
  const uint32_t seed0 = a.have_seed0 ? a.seed0 : 0u;
  ykgpu::render_options ro;
  ro.seed_mode = a.have_seed0 ? YK_SEED_COUNTER : YK_SEED_RANDOM_DEVICE;
  if (a.precision == "fp32") {
    ro.precision = YK_PRECISION_FP32;
  } else if (a.precision != "fp64") {
    std::cerr << "unknown precision " << a.precision << " (fp64|fp32)" << std::endl;
    return EXIT_FAILURE;
  }
  if (a.rng == "xor128") {
    ro.rng = YK_RNG_XOR128;
  } else if (a.rng != "mt19937") {
    std::cerr << "unknown rng " << a.rng << " (mt19937|xor128)" << std::endl;
    return EXIT_FAILURE;
  }
  std::vector<uint8_t> image;
  try {
    ykgpu::renderer gpu(a.device);
    if (!a.scene_file.empty()) {
      uint32_t n = 0;
      yk_camera cam;
      if (yk_scene_read(a.scene_file.c_str(), nullptr, 0, &n, &cam) != YK_OK) {
        std::cerr << "cannot read scene file " << a.scene_file << std::endl;
        return EXIT_FAILURE;
      }
      std::vector<yk_sphere> s(n);
      yk_scene_read(a.scene_file.c_str(), s.data(), n, &n, nullptr);
      gpu.set_records(s, cam);
      if (!a.save_scene.empty()) yk_scene_write(a.save_scene.c_str(), s.data(), n, &cam);
    } else if (a.scene == "ref4") {
      // the reference's world, built with the reference's calls (source.cpp:100-112)
      using T = double;
      using yk::lambertian, yk::metal, yk::pos3, yk::sphere, yk::world_tag;
      const yk::camera<T> cam = {};
      const auto world =
          yk::hittable_list<T>{}
              .add(sphere(pos3<T, world_tag>(0, 0, -1), 0.5, lambertian<double>({0.7, 0.3, 0.3})))
              .add(sphere(pos3<T, world_tag>(0, -100.5, -1), 100.0, lambertian<double>({0.8, 0.8, 0.0})))
              .add(sphere(pos3<T, world_tag>(-1.0, 0.0, -1.0), 0.5, metal<double>({0.8, 0.8, 0.8})))
              .add(sphere(pos3<T, world_tag>(1.0, 0.0, -1.0), 0.5, metal<double>({0.8, 0.6, 0.2})));
      gpu.set_scene(world, cam);
      if (!a.save_scene.empty()) {
        const std::vector<yk_sphere> s = ykgpu::flatten(world);
        const yk_camera c = ykgpu::camera_record(cam);
        yk_scene_write(a.save_scene.c_str(), s.data(), (uint32_t)s.size(), &c);
      }
    } else {
      uint32_t n = 0;
      yk_camera cam;
      if (yk_scene_build(a.scene.c_str(), a.scene_seed, nullptr, 0, &n, &cam) != YK_OK) {
        std::cerr << "unknown scene " << a.scene << std::endl;
        return EXIT_FAILURE;
      }
      std::vector<yk_sphere> s(n);
      yk_scene_build(a.scene.c_str(), a.scene_seed, s.data(), n, &n, nullptr);
      gpu.set_records(s, cam);
      if (!a.save_scene.empty()) yk_scene_write(a.save_scene.c_str(), s.data(), n, &cam);
    }
    std::cout << "rendering..." << std::endl;
    image = gpu.render(W, H, a.spp, a.depth, seed0, ro);
    const yk_render_stats st = gpu.stats();
    if (verbose) {
      ykgpu::render_options vo = ro;
      vo.seed_key = st.seed_key;  // level 3 traces the same samples the image summed
      gpu.print_verbose(std::cout, W, H, a.spp, a.depth, seed0, verbose, vo);
    }
    std::cout << "rendering finished" << std::endl;
    if (a.stats) {
      std::cerr << "kernels " << st.kernel_ms << " ms, " << (double)st.samples / st.kernel_ms / 1e3
                << " Msamples/s, ";
      if (a.have_seed0)
        std::cerr << "seed0 " << seed0 << std::endl;
      else
        std::cerr << "seed key 0x" << std::hex << st.seed_key << std::dec << std::endl;
    }
  } catch (const ykgpu::error& e) {
    std::cerr << e.what() << std::endl;
    return EXIT_FAILURE;
  }

  std::cout << "write to file : " << a.output << std::endl;
  if (!ykpng::write_rgb(a.output.c_str(), W, H, image.data())) {
    std::cout << "error" << std::endl;
    std::exit(EXIT_FAILURE);
  }
  std::cout << "success" << std::endl;
}
