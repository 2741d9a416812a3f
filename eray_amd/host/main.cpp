// eray_main — the reference's example program (src/main.rs:17-78) on the MI355X path:
// load the mesh, build and update main.rs's material graph on the GPU, set up the camera and
// the two lights, render, write the PPM.
//
//   eray_main [--mesh objects/cube.obj] [--width 1024] [--fov 60 60] [--output output.ppm]
//             [--no-debug-dumps]
// Like the reference's debug build, the run also writes rgb.ppm (the rgb node, rgb.rs:96) and
// color.ppm (Material::update, material.rs:41-50) into the working directory.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "eray/eray.hpp"

using namespace eray;
using shader::SocketValue;

int main(int argc, char** argv) {
    std::string mesh = "./objects/cube.obj", output = "output.ppm";
    uint32_t width = 1024;
    float fov_a = 60.0f, fov_b = 60.0f;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--mesh" && i + 1 < argc) mesh = argv[++i];
        else if (a == "--output" && i + 1 < argc) output = argv[++i];
        else if (a == "--width" && i + 1 < argc) width = (uint32_t)std::strtoul(argv[++i], nullptr, 10);
        else if (a == "--no-debug-dumps") set_debug_dumps(false);
        else if (a == "--fov" && i + 2 < argc) {
            fov_a = std::strtof(argv[++i], nullptr);
            fov_b = std::strtof(argv[++i], nullptr);
        } else {
            std::fprintf(stderr, "usage: %s [--mesh PATH] [--width W] [--fov A B] [--output PATH] [--no-debug-dumps]\n", argv[0]);
            return 2;
        }
    }
    try {
        Object<Building> cube = load_obj(mesh);
        if (shader::Status s = shaderlib::example_material(&cube.material)) {
            std::fprintf(stderr, "material: %s\n", s->to_string().c_str());
            return 1;
        }
        // main.rs:22-41
        const std::pair<const char*, float> inputs[] = {{"width", 1024.0f}, {"height", 1024.0f}, {"x_fac", 1.0f},
                                                        {"y_fac", 1.0f},    {"red", 1.0f},      {"green", 0.0f},
                                                        {"blue", 0.0f},     {"factor", 0.5f}};
        for (const auto& [name, v] : inputs)
            if (shader::Status s = cube.material.set_input(name, SocketValue::value(v))) {
                std::fprintf(stderr, "set_input: %s\n", s->to_string().c_str());
                return 1;
            }
        if (shader::Status s = cube.material.update()) {
            std::fprintf(stderr, "update: %s\n", s->to_string().c_str());
            return 1;
        }
        Camera camera;
        camera.center = Vector3(0.0f, 0.0f, 5.0f);
        camera.fov = Fov{fov_a, fov_b};
        camera.width = width;
        Engine engine(camera.size(), 0, 0);  // main.rs:44 with the camera's own size
        Light ambient, point;
        ambient.transform = Transform{}.apply_translation(Vector3(0.0f, 2.0f, 0.0f));
        ambient.variant = LightVariant::Ambient;
        ambient.brightness = 0.2f;
        point.transform = Transform{}.apply_translation(Vector3(1.0f, 1.0f, 2.0f));
        point.variant = LightVariant::Point;
        engine.scene().set_camera(camera).add_light(ambient).add_light(point).add_object(build(std::move(cube)));
        engine.render_to_path(output);
        std::printf("%s: %ux%u\n", output.c_str(), camera.size().first, camera.size().second);
    } catch (const Failure& f) {
        std::fprintf(stderr, "eray status %d: %s\n", f.status, f.what());
        return 1;
    }
    return 0;
}
