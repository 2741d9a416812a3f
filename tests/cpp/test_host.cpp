// Unit tests of the C++ host (include/eray/), mirroring the reference's own tests:
// graph.rs:976-1119 (no_cycle, cycle, macro_validity), shader.rs:181-208
// (shader_function_type), image.rs:201-213 (mod_get), plus the error behaviour of
// validate / set_input / run, the PPM writer and the .obj loader.  `--gpu` adds the device
// parts: the shaderlib nodes through a graph run against eray_material_example, and a render.
//
//   test_host [--gpu] [--root REPO] [--ppm OUT.ppm]
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "eray/eray.hpp"

using namespace eray;
using namespace eray::shader;

static int g_failed = 0, g_run = 0;
#define CHECK(cond)                                                                         \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            std::fprintf(stderr, "  %s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #cond); \
            ++g_failed;                                                                     \
        }                                                                                   \
    } while (0)

static void test(const char* name, const std::function<void()>& fn) {
    ++g_run;
    const int before = g_failed;
    try {
        fn();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "  exception: %s\n", e.what());
        ++g_failed;
    }
    std::printf("%s %s\n", g_failed == before ? "ok  " : "FAIL", name);
}

// graph.rs:982-1010 setup_imports: "identity" = a sub-graph copying its input
static std::map<std::string, ImportedNode<Unvalidated>> setup_imports() {
    GraphNode id;
    id.inputs = {{"value", {std::nullopt, SocketType::Value}}};
    id.outputs = {{"value", SocketValue(SocketType::Value)}};
    id.shader = Shader([](const Sockets& in, Sockets& out) -> ShaderResult {
        ShaderError e;
        const SocketValue* v = get_input(in, "value", SocketType::Value, &e);
        if (!v) return e;
        SocketValue* o = get_output(out, "value", SocketType::Value, &e);
        if (!o) return e;
        o->as_value() = v->as_value().value_or(0.0f);
        return std::nullopt;
    });
    Graph<Unvalidated> g;
    g.inputs = {{"value", SocketValue::value(0.0f)}};
    g.nodes["id"] = Node<Unvalidated>(id);
    g.outputs["value"] = {ssref_node("id", "value"), SocketValue(SocketType::Value)};
    return {{"identity", ImportedNode<Unvalidated>("identity", g)}};
}

static Node<Unvalidated> import_node(const std::map<std::string, ImportedNode<Unvalidated>>& lib, const char* name,
                                     std::optional<SocketRef> value) {
    Node<Unvalidated> n(lib.at(name));
    n.imported().inputs.at("value") = {value, SocketType::IValue};
    return n;
}

static void cpu_tests(const std::string& root) {
    test("graph::cycle_detection::no_cycle", [] {  // graph.rs:1015-1036
        auto imported = setup_imports();
        Graph<Unvalidated> g;
        g.inputs = {{"value", SocketValue(SocketType::IValue)}};
        g.nodes["a"] = import_node(imported, "identity", ssref_graph("value"));
        g.outputs["value"] = {ssref_node("a", "value"), SocketValue(SocketType::IValue)};
        Graph<Validated> v;
        CHECK(!validate(g, &v));
    });
    test("graph::cycle_detection::cycle", [] {  // graph.rs:1038-1072
        auto imported = setup_imports();
        Graph<Unvalidated> g;
        g.nodes["a"] = import_node(imported, "identity", ssref_node("b", "value"));
        g.nodes["b"] = import_node(imported, "identity", ssref_node("a", "value"));
        g.outputs["value"] = {ssref_node("a", "value"), SocketValue(SocketType::IValue)};
        Graph<Validated> v;
        const Status r = validate(g, &v);
        CHECK(r.has_value());
        GraphError expected;
        expected.kind = GraphError::Kind::Cycle;
        expected.detected = "a";
        expected.target_socket = "value";
        expected.source_socket = "value";
        expected.during = {"a", "b"};
        CHECK(r && *r == expected);
    });
    test("graph::macro_validity", [] {  // graph.rs:1075-1118: builder vs field-by-field
        Graph<Unvalidated> manual;
        manual.inputs[Name("iFac")] = SocketValue::value(2.0f);
        GraphNode identity;
        identity.inputs[Name("value")] = {SocketRef::graph("iFac"), SocketType::Value};
        identity.outputs[Name("value")] = SocketValue::value(std::nullopt);
        GraphNode invert;
        invert.inputs[Name("value")] = {SocketRef::of_node("identity", "value"), SocketType::Value};
        invert.outputs[Name("value")] = SocketValue::value(std::nullopt);
        manual.nodes[NodeId("identity")] = Node<Unvalidated>(identity);
        manual.nodes[NodeId("invert")] = Node<Unvalidated>(invert);
        manual.outputs[Name("oFac")] = {SocketRef::of_node("invert", "value"), SocketValue::value(std::nullopt)};

        Graph<Unvalidated> built;
        built.inputs = {{"iFac", SocketValue::value(2.0f)}};
        built.nodes = {{"identity", GraphNode{{{"value", {ssref_graph("iFac"), SocketType::Value}}},
                                              {{"value", SocketValue(SocketType::Value)}},
                                              {}}},
                       {"invert", GraphNode{{{"value", {ssref_node("identity", "value"), SocketType::Value}}},
                                            {{"value", SocketValue(SocketType::Value)}},
                                            {}}}};
        built.outputs = {{"oFac", {ssref_node("invert", "value"), SocketValue::value(std::nullopt)}}};
        CHECK(manual == built);
    });
    test("shader::shader_function_type", [] {  // shader.rs:187-207
        Sockets inputs{{"value", SocketValue(SocketType::Value)}};
        Sockets outputs = inputs;
        bool changed = false;
        const ShaderResult r = Shader([&](const Sockets& in, Sockets& out) -> ShaderResult {
                                   ShaderError e;
                                   const SocketValue* i = get_input(in, "value", SocketType::Value, &e);
                                   if (!i) return e;
                                   SocketValue* o = get_output(out, "value", SocketType::Value, &e);
                                   if (!o) return e;
                                   const auto initial = o->as_value();
                                   o->as_value() = o->as_value().value_or(0.0f) + i->as_value().value_or(0.0f);
                                   changed = initial != o->as_value();
                                   return std::nullopt;
                               }).call(inputs, outputs);
        CHECK(!r);
        CHECK(changed);
    });
    test("shader::get_sv errors", [] {
        Sockets s{{"value", SocketValue(SocketType::IValue)}};
        ShaderError e;
        CHECK(get_input(s, "missing", SocketType::Value, &e) == nullptr);
        CHECK(e.kind == ShaderError::Kind::Missing && e.side == Side::Input && e.names == std::vector<Name>{"missing"});
        CHECK(get_input(s, "value", SocketType::Value, &e) == nullptr);
        CHECK(e.kind == ShaderError::Kind::InvalidType && e.got == SocketType::IValue && e.expected == SocketType::Value);
        CHECK(get_output(s, "nope", SocketType::Value, &e) == nullptr && e.side == Side::Output);
    });
    test("graph: unlinked unset output, missing input", [] {
        Graph<Unvalidated> g;
        g.outputs["out"] = {std::nullopt, SocketValue(SocketType::Value)};
        Graph<Validated> v;
        Status r = validate(g, &v);
        CHECK(r && r->kind == GraphError::Kind::UnlinkedUnsetGraphOutput && r->name == "out");
        g.outputs["out"] = {std::nullopt, SocketValue::value(1.0f)};  // a set output is fine
        CHECK(!validate(g, &v));
        Node<Unvalidated> n(GraphNode{});
        r = n.set_input("absent", ssref_graph("x"));
        CHECK(r && r->kind == GraphError::Kind::Missing && r->side == Side::Input && r->name == "absent");
    });
    test("graph: run through an imported node; set outputs are dropped", [] {
        auto imported = setup_imports();
        {  // the reference's "identity" leaves its inner node unconnected: it always yields 0
            Graph<Unvalidated> g;
            g.inputs = {{"in", SocketValue::value(3.5f)}};
            Node<Unvalidated> a(imported.at("identity"));
            CHECK(!a.set_input("value", ssref_graph("in")));
            g.nodes["a"] = a;
            g.outputs["copy"] = {ssref_node("a", "value"), SocketValue(SocketType::Value)};
            Graph<Validated> v;
            CHECK(!validate(g, &v));
            CHECK(!run(v));
            CHECK(v.outputs.at("copy").second.as_value() == 0.0f);
        }
        // with the inner node wired to the sub-graph's input the value flows through
        auto& inner = *imported.at("identity").inner;
        CHECK(!inner.nodes.at("id").set_input("value", ssref_graph("value")));
        Graph<Unvalidated> g;
        g.inputs = {{"in", SocketValue::value(3.5f)}};
        Node<Unvalidated> a(imported.at("identity"));
        CHECK(!a.set_input("value", ssref_graph("in")));
        g.nodes["a"] = a;
        g.outputs["copy"] = {ssref_node("a", "value"), SocketValue(SocketType::Value)};
        g.outputs["direct"] = {ssref_graph("in"), SocketValue(SocketType::Value)};
        g.outputs["preset"] = {std::nullopt, SocketValue::value(7.0f)};
        Graph<Validated> v;
        CHECK(!validate(g, &v));
        CHECK(!run(v));
        CHECK(v.outputs.count("copy") && v.outputs.at("copy").second.as_value() == 3.5f);
        CHECK(v.outputs.count("direct") && v.outputs.at("direct").second.as_value() == 3.5f);
        CHECK(!v.outputs.count("preset"));  // graph.rs:505
    });
    test("graph: shader errors surface as GraphError::Shader", [] {
        Graph<Unvalidated> g;
        g.nodes["n"] = Node<Unvalidated>(GraphNode{{}, {{"value", SocketValue(SocketType::Value)}},
                                                   Shader([](const Sockets&, Sockets&) -> ShaderResult {
                                                       return ShaderError{ShaderError::Kind::MissingMany,
                                                                          Side::Input,
                                                                          {"width", "height"}};
                                                   })});
        g.outputs["v"] = {ssref_node("n", "value"), SocketValue(SocketType::Value)};
        Graph<Validated> v;
        CHECK(!validate(g, &v));
        const Status r = run(v);
        CHECK(r && r->kind == GraphError::Kind::Shader && r->shader.kind == ShaderError::Kind::MissingMany &&
              r->shader.names == std::vector<Name>({"width", "height"}));
    });
    test("image::mod_get", [] {  // image.rs:201-213
        Image<float> img(10, 10, 0.0f);
        for (size_t i = 0; i < img.pixels.size(); ++i) img.pixels[i] = (float)i;
        CHECK(img.mod_get(123, 12) == img.pixels[2 * 10 + 3]);
    });
    test("image::save_as_ppm bytes", [] {
        Image<Color> img(2, 2, Color());
        img.set(0, 0, Color(1.0f, 0.5f, 0.0f));   // bottom-left: written last
        img.set(1, 1, Color(2.0f, -1.0f, NAN));   // top-right: saturates, NaN -> 0
        const std::vector<uint8_t> b = ppm_bytes(img);
        const std::string header = "P6 2 2 255\n";
        CHECK(b.size() == header.size() + 12);
        CHECK(std::string(b.begin(), b.begin() + header.size()) == header);
        const uint8_t* px = b.data() + header.size();
        CHECK(px[3] == 255 && px[4] == 0 && px[5] == 0);   // row y = 1, x = 1
        CHECK(px[6] == 255 && px[7] == 127 && px[8] == 0);  // row y = 0, x = 0
    });
    test("object::load_obj + build (cube.obj)", [&] {
        Object<Building> o = load_obj(root + "/objects/cube.obj");
        CHECK(o.faces.size() == 12);
        Object<Built> b = build(std::move(o));
        CHECK(b.faces.size() == 12);
    });
    test("object::load_obj errors", [&] {
        const std::string p = "/tmp/eray_host_test.obj";
        auto write = [&](const char* text) {
            FILE* f = std::fopen(p.c_str(), "wb");
            std::fputs(text, f);
            std::fclose(f);
        };
        auto status = [&](const std::function<void()>& fn) {
            try {
                fn();
            } catch (const Failure& e) {
                return e.status;
            }
            return 0;
        };
        write("v 0 0 0\nxyz 1\n");
        CHECK(status([&] { load_obj(p); }) == ERAY_E_PARSE);
        write("v 0 0\n");
        CHECK(status([&] { load_obj(p); }) == ERAY_E_PARSE);
        write("v 0 0 0\nvt 0 0\nf 1/1/1 1/1/1 1/1/1\n");  // normal index past the end: panic
        CHECK(status([&] { load_obj(p); }) == ERAY_E_PARSE);
        write("v 0 0 0\nvt 0 0\n");  // no normals: build's Err
        CHECK(status([&] { build(load_obj(p)); }) == ERAY_E_BUILD);
        CHECK(status([&] { load_obj("/nonexistent/x.obj"); }) == ERAY_E_IO);
        std::remove(p.c_str());
    });
}

static void gpu_tests(const std::string& root, const std::string& ppm) {
    test("shaderlib graph on the GPU == eray_material_example", [] {
        Material m;
        CHECK(!shaderlib::example_material(&m));
        const std::pair<const char*, float> inputs[] = {{"width", 64.0f}, {"height", 32.0f}, {"x_fac", 1.0f},
                                                        {"y_fac", 1.0f},  {"red", 1.0f},     {"green", 0.0f},
                                                        {"blue", 0.0f},   {"factor", 0.5f}};
        for (const auto& [n, v] : inputs) CHECK(!m.set_input(n, SocketValue::value(v)));
        CHECK(!m.update());
        const auto& outs = m.graph().outputs;
        CHECK(outs.count("color") && outs.count("diffuse"));
        const Image<Color> color = outs.at("color").second.as_icolor()->to_host();
        const Image<float> diffuse = outs.at("diffuse").second.as_ivalue()->to_host();
        DeviceImage<Color> rc(64, 32);
        DeviceImage<float> rd(64, 32);
        Device& d = Device::current();
        d.check(eray_material_example(d.ctx(), 64, 32, 1.0f, 1.0f, 1.0f, 0.0f, 0.0f, 0.5f,
                                      reinterpret_cast<float*>(rc.data()), rd.data()));
        CHECK(color == rc.to_host());
        CHECK(diffuse == rd.to_host());
    });
    test("shaderlib: missing inputs -> MissingMany", [] {
        shaderlib::GraphResult g;
        CHECK(!shaderlib::wave::graph(&g));
        Graph<Validated> v;
        CHECK(!validate(g, &v));
        const Status r = run(v);  // width / height unset
        CHECK(r && r->kind == GraphError::Kind::Shader && r->shader.kind == ShaderError::Kind::MissingMany &&
              r->shader.names == std::vector<Name>({"width", "height"}));
    });
    test("engine: main.rs scene at 256x256 (PPM written for the golden check)", [&] {
        Object<Building> cube = load_obj(root + "/objects/cube.obj");
        CHECK(!shaderlib::example_material(&cube.material));
        const std::pair<const char*, float> inputs[] = {{"width", 1024.0f}, {"height", 1024.0f}, {"x_fac", 1.0f},
                                                        {"y_fac", 1.0f},    {"red", 1.0f},      {"green", 0.0f},
                                                        {"blue", 0.0f},     {"factor", 0.5f}};
        for (const auto& [n, v] : inputs) CHECK(!cube.material.set_input(n, SocketValue::value(v)));
        CHECK(!cube.material.update());
        Camera cam;
        cam.center = Vector3(0.0f, 0.0f, 5.0f);
        cam.fov = Fov{60.0f, 60.0f};
        cam.width = 256;
        Engine engine({256, 256}, 0, 0);
        Light amb, pt;
        amb.transform = Transform{}.apply_translation(Vector3(0.0f, 2.0f, 0.0f));
        amb.variant = LightVariant::Ambient;
        amb.brightness = 0.2f;
        pt.transform = Transform{}.apply_translation(Vector3(1.0f, 1.0f, 2.0f));
        engine.scene().set_camera(cam).add_light(amb).add_light(pt).add_object(build(std::move(cube)));
        const Image<Color>& img = engine.render_to_path(ppm);
        // the survey's centre pixel: face 1, RGB ~ (0.548175, 0.311178, 0.311178)
        const Color c = img.pixels[(size_t)128 * 256 + 128];
        CHECK(std::fabs(c.r - 0.548175f) < 2e-6f && std::fabs(c.g - 0.311178f) < 2e-6f);
    });
}

int main(int argc, char** argv) {
    bool gpu = false;
    std::string root = ".", ppm = "/tmp/eray_host_c1.ppm";
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--gpu")) gpu = true;
        else if (!std::strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
        else if (!std::strcmp(argv[i], "--ppm") && i + 1 < argc) ppm = argv[++i];
    }
    cpu_tests(root);
    if (gpu) gpu_tests(root, ppm);
    std::printf("%d tests, %d failed checks\n", g_run, g_failed);
    return g_failed ? 1 : 0;
}
