// engine.cpp — Camera, Material, Object (load_obj / build), Scene and Engine of the C++ host
// (src/lib/{camera,material,object,scene,engine}.rs), rendering through the C-ABI.
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>

#include "eray/engine.hpp"

namespace eray {

using namespace shader;

// camera.rs:36-38
std::pair<uint32_t, uint32_t> Camera::size() const {
    eray_camera c{{center.x, center.y, center.z}, {fov.a, fov.b}, width, z_dist};
    uint32_t w = 0, h = 0;
    eray_camera_size(&c, &w, &h);
    return {w, h};
}

// ---------------------------------------------------------------------------- Material -----
Material::Material(Graph<Validated> graph, std::map<StandardMaterialOutput, Name> selected)
    : selected_(std::move(selected)), graph_(std::move(graph)), recompute_(true) {}

Status Material::update() {  // material.rs:35-53
    if (recompute_) {
        if (Status s = run(graph_)) return s;
        recompute_ = false;
    }
    // material.rs:41-50 (#[cfg(debug_assertions)]): the Color output's image to color.ppm (the
    // reference panics when that output is not an IColor)
    if (debug_dumps()) {
        auto sel = selected_.find(StandardMaterialOutput::Color);
        if (sel != selected_.end()) {
            auto out = graph_.outputs.find(sel->second);
            if (out != graph_.outputs.end()) {
                const SocketValue& v = out->second.second;
                if (v.type() != SocketType::IColor) throw Failure(ERAY_E_INVALID_TYPE, "color output is not an IColor");
                if (v.as_icolor()) save_as_ppm(v.as_icolor()->to_host(), "color.ppm");
            }
        }
    }
    return std::nullopt;
}

Status Material::set_input(const Name& name, SocketValue value) {  // material.rs:96-104
    auto it = graph_.inputs.find(name);
    if (it == graph_.inputs.end()) {
        GraphError e;
        e.kind = GraphError::Kind::Missing;
        e.side = Side::Input;
        e.name = name;
        return e;
    }
    it->second = std::move(value);
    return std::nullopt;
}

eray_material Material::device_material() const {  // Material::get's selection (material.rs:56-94)
    eray_material m{};
    auto image = [&](StandardMaterialOutput o, SocketType kind) {
        eray_image none{nullptr, 0, 0};
        auto sel = selected_.find(o);
        if (sel == selected_.end()) return none;
        auto out = graph_.outputs.find(sel->second);
        if (out == graph_.outputs.end()) return none;
        const SocketValue& v = out->second.second;
        if (v.type() != kind) return none;  // other kinds are ignored (None)
        if (kind == SocketType::IColor) return v.as_icolor() ? v.as_icolor()->view() : none;
        return v.as_ivalue() ? v.as_ivalue()->view() : none;
    };
    m.color = image(StandardMaterialOutput::Color, SocketType::IColor);
    m.diffuse = image(StandardMaterialOutput::Diffuse, SocketType::IValue);
    m.specular = image(StandardMaterialOutput::Specular, SocketType::IValue);
    m.specular_power = image(StandardMaterialOutput::SpecularPower, SocketType::IValue);
    m.reflection = image(StandardMaterialOutput::Reflection, SocketType::IValue);
    return m;
}

// ----------------------------------------------------------------------------- .obj --------
namespace {
[[noreturn]] void parse_panic(const std::string& what) { throw Failure(ERAY_E_PARSE, what); }

// Rust's str::parse::<f32>: decimal / exponent forms and inf / infinity / nan (any case),
// correctly rounded (strtof)
float parse_f32(const std::string& t) {
    const char* s = t.c_str();
    size_t i = (s[0] == '+' || s[0] == '-') ? 1 : 0;
    std::string rest = t.substr(i);
    for (auto& c : rest) c = (char)std::tolower((unsigned char)c);
    bool ok = rest == "inf" || rest == "infinity" || rest == "nan";
    if (!ok) {  // digits [. digits] [e [+-] digits] with at least one digit in the mantissa
        size_t k = 0, digits = 0;
        while (k < rest.size() && std::isdigit((unsigned char)rest[k])) ++k, ++digits;
        if (k < rest.size() && rest[k] == '.') {
            ++k;
            while (k < rest.size() && std::isdigit((unsigned char)rest[k])) ++k, ++digits;
        }
        ok = digits > 0;
        if (ok && k < rest.size() && rest[k] == 'e') {
            ++k;
            if (k < rest.size() && (rest[k] == '+' || rest[k] == '-')) ++k;
            size_t e = 0;
            while (k < rest.size() && std::isdigit((unsigned char)rest[k])) ++k, ++e;
            ok = e > 0;
        }
        ok = ok && k == rest.size();
    }
    if (!ok) parse_panic("Failed to parse coords, should be an f32: " + t);
    if (rest == "nan") return std::nanf("");
    return std::strtof(s, nullptr);
}

// object.rs:396-413
std::vector<float> parse_coords(std::istringstream& tokens, size_t line) {
    std::vector<float> c;
    std::string t;
    while (tokens >> t) c.push_back(parse_f32(t));
    if (c.size() < 2 || c.size() >= 4)
        parse_panic("Invalid coordinate count at line " + std::to_string(line));
    return c;
}

// object.rs:415-421: "a/b/c" -> Option<usize> each
std::vector<std::optional<size_t>> parse_indices(const std::string& s) {
    std::vector<std::optional<size_t>> r;
    size_t start = 0;
    while (true) {
        const size_t slash = s.find('/', start);
        const std::string part = s.substr(start, slash == std::string::npos ? std::string::npos : slash - start);
        std::optional<size_t> v;
        std::string digits = !part.empty() && part[0] == '+' ? part.substr(1) : part;
        if (!digits.empty() && digits.find_first_not_of("0123456789") == std::string::npos && digits.size() < 20)
            v = (size_t)std::strtoull(digits.c_str(), nullptr, 10);
        r.push_back(v);
        if (slash == std::string::npos) break;
        start = slash + 1;
    }
    return r;
}
}  // namespace

Object<Building> load_obj(const std::string& path) {  // object.rs:101-186
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Failure(ERAY_E_IO, "cannot read " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string content = ss.str();
    Object<Building> obj;
    std::vector<Vector3>& vertices = obj.vertices;
    std::vector<Vector3>& normals = obj.normals;
    std::vector<std::array<float, 2>>& uvs = obj.uvs;
    size_t line = 0, pos = 0;
    while (pos <= content.size()) {  // str::lines(): \n or \r\n separated
        size_t end = content.find('\n', pos);
        if (end == std::string::npos) end = content.size();
        std::string l = content.substr(pos, end - pos);
        if (!l.empty() && l.back() == '\r') l.pop_back();
        const bool last = end == content.size();
        pos = end + 1;
        const size_t lineno = line++;
        if (last && l.empty()) break;
        if (l.empty() || l[0] == '#') continue;
        std::istringstream tokens(l);
        std::string marker;
        if (!(tokens >> marker)) parse_panic("empty line " + std::to_string(lineno));  // unwrap on None
        if (marker == "o" || marker == "g") {
            std::string name;
            if (!(tokens >> name)) parse_panic("missing name at line " + std::to_string(lineno));
        } else if (marker == "s") {
            std::string v;
            if (!(tokens >> v)) parse_panic("missing smooth shading value at line " + std::to_string(lineno));
            if (v != "1" && v != "on" && v != "0" && v != "off") parse_panic("Unhandled smooth shading setting `" + v + "`");
        } else if (marker == "v" || marker == "vn") {
            const std::vector<float> c = parse_coords(tokens, lineno);
            if (c.size() < 3) parse_panic("coordinate count at line " + std::to_string(lineno));  // coords[0..=2]
            (marker == "v" ? vertices : normals).push_back(Vector3(c[0], c[1], c[2]));
        } else if (marker == "vt") {
            const std::vector<float> c = parse_coords(tokens, lineno);
            uvs.push_back({c[0], c[1]});
        } else if (marker == "f") {
            std::vector<std::array<size_t, 3>> verts;
            std::string tok;
            while (tokens >> tok) {
                const auto idx = parse_indices(tok);
                if (idx.size() < 3 || !idx[0] || !idx[1] || !idx[2]) parse_panic("face index at line " + std::to_string(lineno));
                const size_t a = *idx[0], b = *idx[1], c = *idx[2];
                if (a == 0 || b == 0 || c == 0 || a > vertices.size() || b > uvs.size() || c > normals.size())
                    parse_panic("face index out of range at line " + std::to_string(lineno));
                verts.push_back({a - 1, b - 1, c - 1});
            }
            if (verts.size() != 3)
                parse_panic("Invalid vertex count for face at line " + std::to_string(lineno) + " (should be 3, is " +
                            std::to_string(verts.size()) + ")");
            Triangle t;
            for (int k = 0; k < 3; ++k) {
                t.pos[k] = vertices[verts[k][0]];
                t.uv[k] = uvs[verts[k][1]];
                t.normal[k] = normals[verts[k][2]];
            }
            obj.faces.push_back(t);
        } else {
            parse_panic("Unhandled marker " + marker);
        }
    }
    obj.bbox = {Vector3(), Vector3()};  // BoundingBox::default (object.rs:306-315)
    return obj;
}

Object<Built> build(Object<Building> object) {  // object.rs:213-230
    if (object.vertices.empty()) throw Failure(ERAY_E_BUILD, "Missing vertices");
    if (object.normals.empty()) throw Failure(ERAY_E_BUILD, "Missing normals");
    Object<Built> b;
    b.vertices = std::move(object.vertices);
    b.normals = std::move(object.normals);
    b.uvs = std::move(object.uvs);
    b.faces = std::move(object.faces);
    b.bbox = object.bbox;
    b.material = std::move(object.material);
    return b;
}

// ------------------------------------------------------------------------------- Scene -----
Scene& Scene::set_camera(Camera camera) {
    camera_ = camera;
    dirty_ = true;
    return *this;
}
Scene& Scene::add_light(Light light) {
    lights_.push_back(light);
    dirty_ = true;
    return *this;
}
Scene& Scene::add_object(Object<Built> object) {
    objects_.push_back(std::move(object));
    dirty_ = true;
    return *this;
}

// ------------------------------------------------------------------------------ Engine -----
Engine::Engine(std::pair<uint32_t, uint32_t> size, uint32_t bounces, uint32_t anti_aliasing)
    : image_(size.first, size.second, Color()), bounces_(bounces), anti_aliasing_(anti_aliasing) {
    // rand::thread_rng is seeded from the OS (engine.rs:49): so is the jitter stream by default
    std::random_device rd;
    aa_seed_ = ((uint64_t)rd() << 32) | rd();
}

void Engine::upload() {
    Device& d = Device::current();
    eray_ctx* c = d.ctx();
    d.check(eray_scene_reset(c));
    const Camera& cam = scene_.camera_;
    eray_camera ec{{cam.center.x, cam.center.y, cam.center.z}, {cam.fov.a, cam.fov.b}, cam.width, cam.z_dist};
    d.check(eray_scene_set_camera(c, &ec));
    for (const Light& l : scene_.lights_) {
        const eray_light el{{l.transform.translation.x, l.transform.translation.y, l.transform.translation.z},
                            l.variant == LightVariant::Ambient ? ERAY_LIGHT_AMBIENT : ERAY_LIGHT_POINT,
                            {l.color.r, l.color.g, l.color.b},
                            l.brightness};
        d.check(eray_scene_add_light(c, &el));
    }
    for (Object<Built>& o : scene_.objects_) {
        const size_t T = o.faces.size();
        std::vector<float> pos(9 * T), nrm(9 * T), uv(6 * T);
        for (size_t i = 0; i < T; ++i)
            for (int k = 0; k < 3; ++k) {
                const Triangle& t = o.faces[i];
                pos[9 * i + 3 * k + 0] = t.pos[k].x;
                pos[9 * i + 3 * k + 1] = t.pos[k].y;
                pos[9 * i + 3 * k + 2] = t.pos[k].z;
                nrm[9 * i + 3 * k + 0] = t.normal[k].x;
                nrm[9 * i + 3 * k + 1] = t.normal[k].y;
                nrm[9 * i + 3 * k + 2] = t.normal[k].z;
                uv[6 * i + 2 * k + 0] = t.uv[k][0];
                uv[6 * i + 2 * k + 1] = t.uv[k][1];
            }
        eray_object eo{};
        eo.positions = pos.data();
        eo.normals = nrm.data();
        eo.uvs = uv.data();
        eo.triangle_count = (uint32_t)T;
        eo.bbox_min[0] = o.bbox[0].x, eo.bbox_min[1] = o.bbox[0].y, eo.bbox_min[2] = o.bbox[0].z;
        eo.bbox_max[0] = o.bbox[1].x, eo.bbox_max[1] = o.bbox[1].y, eo.bbox_max[2] = o.bbox[1].z;
        eo.material = o.material.device_material();
        d.check(eray_scene_add_object(c, &eo, nullptr));
    }
    scene_.dirty_ = false;
}

const Image<Color>& Engine::render() {  // engine.rs:46-81
    Device& d = Device::current();
    if (scene_.dirty_) upload();
    const size_t n = (size_t)image_.width * image_.height;
    if (!rgb_ || rgb_->size() < 12 * n) rgb_ = std::make_shared<DeviceBuffer>(12 * n);
    // Image::set writes pixels the camera covers; the rest keep the engine's initial black
    d.check(eray_memset(d.ctx(), rgb_->data(), 0, 12 * n));
    const uint32_t h = scene_.camera_.size().second;
    eray_render_params p{image_.width, image_.height, 0, h, bounces_, anti_aliasing_,
                         static_cast<float*>(rgb_->data()), nullptr, nullptr, ERAY_RENDER_DEFAULT, aa_seed_};
    d.check(eray_render(d.ctx(), &p));
    d.check(eray_copy_to_host(d.ctx(), image_.pixels.data(), rgb_->data(), 12 * n));
    return image_;
}

const Image<Color>& Engine::render_to_path(const std::string& path) {  // engine.rs:86-98
    render();
    save_as_ppm(image_, path);
    return image_;
}

}  // namespace eray
