// oracle/ref_dropin.cpp — drop-in demonstration (test infrastructure; built into oracle/_ref/
// only where /root/reference exists, then run on the GPU box by tests/test_cli.py).
//
// Compiles the reference's OWN scene types (/root/reference/yk/{hittable_list,sphere,material,
// camera}.hpp, included in place) and hands its world — built exactly as render() builds it,
// source.cpp:100-112 — to the GPU through include/yk/ykgpu_bridge.hpp and the C-ABI, in place
// of the for_each loop of source.cpp:122-172.  This is the change INTEGRATION.md shows for
// source.cpp itself.  Writes the image_t bytes (W*H*3) to argv[1].
//   usage: ref_dropin out.rgb W spp depth seed0
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "yk/camera.hpp"
#include "yk/color.hpp"
#include "yk/config.hpp"
#include "yk/hittable.hpp"
#include "yk/hittable_list.hpp"
#include "yk/material.hpp"
#include "yk/sphere.hpp"
#include "yk/vec3.hpp"
// ours (found through -I include/, after the reference's yk/ directory)
#include "yk/ykgpu_bridge.hpp"

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s out.rgb W spp depth seed0\n", argv[0]);
    return 2;
  }
  const uint32_t W = std::strtoul(argv[2], nullptr, 10), spp = std::strtoul(argv[3], nullptr, 10);
  const uint32_t depth = std::strtoul(argv[4], nullptr, 10), seed0 = std::strtoul(argv[5], nullptr, 10);
  const uint32_t H = static_cast<uint32_t>(W / (16.0 / 9.0));  // source.cpp:61-62

  // render()'s own declarations, source.cpp:100-112, reference types
  using namespace yk;
  using T = double;
  using color = color3d;
  const camera<T> cam = {};
  const auto world =
      hittable_list<T>{}
          .add(sphere(pos3<T, world_tag>(0, 0, -1), 0.5, lambertian<color::value_type>({0.7, 0.3, 0.3})))
          .add(sphere(pos3<T, world_tag>(0, -100.5, -1), 100.0, lambertian<color::value_type>({0.8, 0.8, 0.0})))
          .add(sphere(pos3<T, world_tag>(-1.0, 0.0, -1.0), 0.5, metal<color::value_type>({0.8, 0.8, 0.8})))
          .add(sphere(pos3<T, world_tag>(1.0, 0.0, -1.0), 0.5, metal<color::value_type>({0.8, 0.6, 0.2})));

  try {
    ykgpu::renderer gpu;
    gpu.set_scene(world, cam);
    const std::vector<uint8_t> img = gpu.render(W, H, spp, depth, seed0);
    FILE* f = std::fopen(argv[1], "wb");
    if (!f) return 1;
    std::fwrite(img.data(), 1, img.size(), f);
    std::fclose(f);
  } catch (const ykgpu::error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
