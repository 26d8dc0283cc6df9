// rt_ref_adapter.hpp — the reference-side binding of the MI355X path.
//
// Code a maintainer adds to alp-aydin/Raytracing-Project (it includes the
// reference's own headers): it walks an API-built or JSON-loaded
// Scene + Camera (raytracer/src/scene.h:32-67, camera.h:26-79) into the
// C-ABI's scene IR (include/rt.h rt_scene_desc) so that Tracer::render
// (tracer.h:18-35, tracer.cpp:247-305) can delegate to rt_render_multi - no
// JSON re-parse, directional lights included (scene.h:10-15, shading.cpp:46-76).
// See INTEGRATION.md for the Tracer::render body that uses it.
#pragma once

#include <vector>

#include "camera.h"
#include "core.h"
#include "scene.h"
#include "rt.h"

namespace rtref {

// Build an rt_scene (owned by the caller: rt_scene_destroy) from the
// reference objects.  Material identity is kept by POINTER (the paper-mode
// edge test compares Material pointers, tracer.cpp:170): every distinct
// Material* becomes one IR material, each Pokeball's five region materials
// included.  Returns an rt_status; on failure rt_last_error() explains.
int scene_from_reference(const Scene& scene, const Camera& cam, rt_scene** out);

// Tracer::render on n_gpus GPUs of this process (0 = all visible): converts
// the scene, renders into fb (resized to W*H, top row first, exactly like
// the reference), and throws std::runtime_error on a device error.
void render_on_gpu(const Scene& scene, const Camera& cam, int width, int height, bool paper,
                   std::vector<Color>& framebuffer, int n_gpus = 0);

}  // namespace rtref
