// engine.hpp — the render side of the C++ host: Vector, Camera, Light, Material, Object,
// Scene and Engine with the reference's builder API (src/lib/{camera,light,material,object,
// scene,engine}.rs), rendering through the C-ABI (include/eray_hip.h) on the current Device.
#pragma once

#include <array>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "graph.hpp"
#include "image.hpp"

namespace eray {

struct Vector3 {
    float x = 0.0f, y = 0.0f, z = 0.0f;
    Vector3() = default;
    Vector3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
};

struct Fov {  // camera.rs:8-12 Fov(f32, f32)
    float a = 60.0f, b = 60.0f;
    float ratio() const { return a / b; }
};

// camera.rs:15-38 (target / up are not used by the render path)
struct Camera {
    Vector3 center{0.0f, 0.0f, 0.0f};
    Fov fov{60.0f, 60.0f};
    uint32_t width = 1024;
    float z_dist = 1.0f;
    // camera.rs:36-38: (width, (width as f32 / fov.ratio()) as u32)
    std::pair<uint32_t, uint32_t> size() const;
};

struct Transform {  // transform.rs: only the translation reaches the path
    Vector3 translation;
    Transform apply_translation(Vector3 t) const { return Transform{t}; }
};

enum class LightVariant { Point, Ambient };  // light.rs:20-25

struct Light {  // light.rs:7-16
    Transform transform;
    LightVariant variant = LightVariant::Point;
    Color color{1.0f, 1.0f, 1.0f};
    float brightness = 1.0f;
};

// material.rs:96-104
enum class StandardMaterialOutput { Color, Diffuse, Specular, SpecularPower, Reflection };

// material.rs:13-94: a validated graph and the outputs that feed the renderer
class Material {
public:
    Material() = default;
    Material(shader::Graph<shader::Validated> graph, std::map<StandardMaterialOutput, shader::Name> selected);
    // material.rs:35-53: runs the graph once (until an input changes)
    shader::Status update();
    // material.rs:96-112: set a graph input (Missing(Input, name) if absent)
    shader::Status set_input(const shader::Name& name, shader::SocketValue value);
    // the selected outputs as device images (IColor for Color, IValue for the others; any
    // other kind is ignored, as Material::get does)
    eray_material device_material() const;
    const shader::Graph<shader::Validated>& graph() const { return graph_; }

private:
    std::map<StandardMaterialOutput, shader::Name> selected_;
    shader::Graph<shader::Validated> graph_;
    bool recompute_ = true;
};

struct Building {};  // object.rs typestate
struct Built {};

struct Triangle {  // primitives.rs: positions, vertex normals, uvs of a face
    std::array<Vector3, 3> pos, normal;
    std::array<std::array<float, 2>, 3> uv;
};

// object.rs:30-52
template <class State>
struct Object {
    std::vector<Vector3> vertices, normals;
    std::vector<std::array<float, 2>> uvs;
    std::vector<Triangle> faces;
    std::array<Vector3, 2> bbox{};  // (0,0,0)-(0,0,0) for loaded meshes (object.rs:306-315)
    Material material;
};

// object.rs:101-186 Object::load_obj (the reference's dialect; its panics become Failure with
// ERAY_E_PARSE / ERAY_E_IO)
Object<Building> load_obj(const std::string& path);
// object.rs:213-230 Object::build: "Missing vertices" / "Missing normals" -> Failure with
// ERAY_E_BUILD
Object<Built> build(Object<Building> object);

// scene.rs:12-54
class Scene {
public:
    Scene& set_camera(Camera camera);
    Scene& add_light(Light light);
    Scene& add_object(Object<Built> object);
    const Camera& camera() const { return camera_; }
    std::vector<Object<Built>>& objects() { return objects_; }
    const std::vector<Light>& lights() const { return lights_; }

private:
    Camera camera_{};
    std::vector<Light> lights_;
    std::vector<Object<Built>> objects_;
    friend class Engine;
    bool dirty_ = true;
};

// engine.rs:13-98
class Engine {
public:
    // Engine::new((width, height), bounces, anti_aliasing)
    Engine(std::pair<uint32_t, uint32_t> size, uint32_t bounces, uint32_t anti_aliasing);
    Scene& scene() { scene_.dirty_ = true; return scene_; }
    // engine.rs:46-81: renders on the GPU; the f32 image (Image<Color>) is copied back
    const Image<Color>& render();
    // engine.rs:86-98: render + save_as_ppm (the PPM bytes come from the device, fused)
    const Image<Color>& render_to_path(const std::string& path);
    // The anti-aliasing jitter stream's key (eray_render_params::aa_seed).  The reference draws
    // from the OS-seeded thread_rng; a new Engine picks a random seed likewise, and fixing it
    // makes anti-aliased renders reproducible.
    void set_aa_seed(uint64_t seed) { aa_seed_ = seed; }
    uint64_t aa_seed() const { return aa_seed_; }

private:
    void upload();
    Image<Color> image_;
    Scene scene_;
    uint32_t bounces_, anti_aliasing_;
    uint64_t aa_seed_ = 0;
    std::shared_ptr<DeviceBuffer> rgb_, ppm_;
};

}  // namespace eray
