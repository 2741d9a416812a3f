// shaderlib.cpp — src/shaderlib/{wave,rgb,flat_color,mix_color}.rs and main.rs's material on
// the C++ host: the node bodies call the C-ABI node operators on the current Device.
#include "eray/shaderlib.hpp"

namespace eray {
namespace shaderlib {

using namespace shader;

namespace {

uint32_t sat_u32(float f) {  // Rust's `f as u32`
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}

// get_sv! + handle_missing_socket_values! (shaderlib/utils.rs:1-35) in one place
struct Args {
    const Sockets& in;
    ShaderError err;
    bool failed = false;
    std::vector<Name> missing;

    const SocketValue* get(const char* name, SocketType kind) {
        if (failed) return nullptr;
        const SocketValue* v = get_input(in, name, kind, &err);
        failed = v == nullptr;
        return v;
    }
    void need(const char* name, const SocketValue* v) {
        if (v && v->is_none()) missing.push_back(name);
    }
    ShaderResult missing_error() const {
        if (missing.empty()) return std::nullopt;
        return ShaderError{ShaderError::Kind::MissingMany, Side::Input, missing};
    }
};

GraphNode make_node(NodeInputs inputs, Sockets outputs, Shader::Fn fn) {
    GraphNode n;
    n.inputs = std::move(inputs);
    n.outputs = std::move(outputs);
    n.shader = Shader(std::move(fn));
    return n;
}

Status connect(Node<Unvalidated>& node, std::initializer_list<std::pair<const char*, std::optional<SocketRef>>> links) {
    for (const auto& [name, ref] : links)
        if (Status s = node.set_input(name, ref)) return s;
    return std::nullopt;
}

}  // namespace

namespace wave {
// wave.rs:100-137
NodeResult node() {
    return make_node({{"width", {std::nullopt, SocketType::Value}},
                      {"height", {std::nullopt, SocketType::Value}},
                      {"x_fac", {std::nullopt, SocketType::Value}},
                      {"y_fac", {std::nullopt, SocketType::Value}}},
                     {{"value", SocketValue(SocketType::IValue)}},
                     [](const Sockets& inputs, Sockets& outputs) -> ShaderResult {
                         Args a{inputs};
                         const SocketValue* width = a.get("width", SocketType::Value);
                         const SocketValue* height = a.get("height", SocketType::Value);
                         const SocketValue* x_fac = a.get("x_fac", SocketType::Value);
                         const SocketValue* y_fac = a.get("y_fac", SocketType::Value);
                         if (a.failed) return a.err;
                         ShaderError e;
                         SocketValue* out = get_output(outputs, "value", SocketType::IValue, &e);
                         if (!out) return e;
                         a.need("width", width);
                         a.need("height", height);
                         if (ShaderResult m = a.missing_error()) return m;
                         const float xf = x_fac->as_value().value_or(DEFAULT_FACTOR);
                         const float yf = y_fac->as_value().value_or(DEFAULT_FACTOR);
                         DeviceImage<float> res(sat_u32(*width->as_value()), sat_u32(*height->as_value()));
                         Device& d = Device::current();
                         d.check(eray_node_wave(d.ctx(), res.width, res.height, xf, yf, res.data()));
                         out->as_ivalue() = res;
                         return std::nullopt;
                     });
}

Status graph(GraphResult* out) {  // wave.rs:76-98
    GraphResult g;
    g.inputs = {{"width", SocketValue(SocketType::Value)},
                {"height", SocketValue(SocketType::Value)},
                {"x_fac", SocketValue::value(DEFAULT_FACTOR)},
                {"y_fac", SocketValue::value(DEFAULT_FACTOR)}};
    NodeResult n = node();
    if (Status s = connect(n, {{"width", ssref_graph("width")},
                               {"height", ssref_graph("height")},
                               {"x_fac", ssref_graph("x_fac")},
                               {"y_fac", ssref_graph("y_fac")}}))
        return s;
    g.nodes["wave"] = std::move(n);
    g.outputs["value"] = {ssref_node("wave", "value"), SocketValue(SocketType::Value)};
    *out = std::move(g);
    return std::nullopt;
}
}  // namespace wave

namespace rgb {
// rgb.rs:64-103
NodeResult node() {
    return make_node({{"width", {std::nullopt, SocketType::Value}},
                      {"height", {std::nullopt, SocketType::Value}},
                      {"red", {std::nullopt, SocketType::IValue}},
                      {"green", {std::nullopt, SocketType::IValue}},
                      {"blue", {std::nullopt, SocketType::IValue}}},
                     {{"color", SocketValue(SocketType::IColor)}},
                     [](const Sockets& inputs, Sockets& outputs) -> ShaderResult {
                         Args a{inputs};
                         const SocketValue* width = a.get("width", SocketType::Value);
                         const SocketValue* height = a.get("height", SocketType::Value);
                         const SocketValue* red = a.get("red", SocketType::IValue);
                         const SocketValue* green = a.get("green", SocketType::IValue);
                         const SocketValue* blue = a.get("blue", SocketType::IValue);
                         if (a.failed) return a.err;
                         ShaderError e;
                         SocketValue* out = get_output(outputs, "color", SocketType::IColor, &e);
                         if (!out) return e;
                         a.need("width", width);
                         a.need("height", height);
                         a.need("red", red);
                         a.need("green", green);
                         a.need("blue", blue);
                         if (ShaderResult m = a.missing_error()) return m;
                         DeviceImage<Color> res(sat_u32(*width->as_value()), sat_u32(*height->as_value()));
                         Device& d = Device::current();
                         d.check(eray_node_rgb(d.ctx(), res.width, res.height, red->as_ivalue()->view(),
                                               green->as_ivalue()->view(), blue->as_ivalue()->view(),
                                               reinterpret_cast<float*>(res.data())));
                         // rgb.rs:96: the node writes its image to rgb.ppm in the working directory
                         if (debug_dumps()) save_as_ppm(res.to_host(), "rgb.ppm");
                         out->as_icolor() = res;
                         return std::nullopt;
                     });
}

Status graph(GraphResult* out) {  // rgb.rs:39-62
    GraphResult g;
    g.inputs = {{"width", SocketValue(SocketType::Value)},
                {"height", SocketValue(SocketType::Value)},
                {"red", SocketValue(SocketType::IValue)},
                {"green", SocketValue(SocketType::IValue)},
                {"blue", SocketValue(SocketType::IValue)}};
    NodeResult n = node();
    if (Status s = connect(n, {{"width", ssref_graph("width")},
                               {"height", ssref_graph("height")},
                               {"red", ssref_graph("red")},
                               {"green", ssref_graph("green")},
                               {"blue", ssref_graph("blue")}}))
        return s;
    g.nodes["converter"] = std::move(n);
    g.outputs["color"] = {ssref_node("converter", "color"), SocketValue(SocketType::IColor)};
    *out = std::move(g);
    return std::nullopt;
}
}  // namespace rgb

namespace flat_color {
// flat_color.rs:65-95
NodeResult node() {
    return make_node({{"width", {std::nullopt, SocketType::Value}},
                      {"height", {std::nullopt, SocketType::Value}},
                      {"red", {std::nullopt, SocketType::Value}},
                      {"green", {std::nullopt, SocketType::Value}},
                      {"blue", {std::nullopt, SocketType::Value}}},
                     {{"color", SocketValue(SocketType::IColor)}},
                     [](const Sockets& inputs, Sockets& outputs) -> ShaderResult {
                         Args a{inputs};
                         const SocketValue* width = a.get("width", SocketType::Value);
                         const SocketValue* height = a.get("height", SocketType::Value);
                         const SocketValue* red = a.get("red", SocketType::Value);
                         const SocketValue* green = a.get("green", SocketType::Value);
                         const SocketValue* blue = a.get("blue", SocketType::Value);
                         if (a.failed) return a.err;
                         ShaderError e;
                         SocketValue* out = get_output(outputs, "color", SocketType::IColor, &e);
                         if (!out) return e;
                         a.need("width", width);
                         a.need("height", height);
                         a.need("red", red);
                         a.need("green", green);
                         a.need("blue", blue);
                         if (ShaderResult m = a.missing_error()) return m;
                         DeviceImage<Color> res(sat_u32(*width->as_value()), sat_u32(*height->as_value()));
                         Device& d = Device::current();
                         d.check(eray_node_flat_color(d.ctx(), res.width, res.height, *red->as_value(),
                                                      *green->as_value(), *blue->as_value(),
                                                      reinterpret_cast<float*>(res.data())));
                         out->as_icolor() = res;
                         return std::nullopt;
                     });
}

Status graph(GraphResult* out) {  // flat_color.rs:39-63
    GraphResult g;
    g.inputs = {{"red", SocketValue(SocketType::Value)},
                {"green", SocketValue(SocketType::Value)},
                {"blue", SocketValue(SocketType::Value)},
                {"width", SocketValue::value(1.0f)},
                {"height", SocketValue::value(1.0f)}};
    NodeResult n = node();
    if (Status s = connect(n, {{"width", ssref_graph("width")},
                               {"height", ssref_graph("height")},
                               {"red", ssref_graph("red")},
                               {"green", ssref_graph("green")},
                               {"blue", ssref_graph("blue")}}))
        return s;
    g.nodes["converter"] = std::move(n);
    g.outputs["color"] = {ssref_node("converter", "color"), SocketValue(SocketType::IColor)};
    *out = std::move(g);
    return std::nullopt;
}
}  // namespace flat_color

namespace mix_color {
// mix_color.rs:57-102 (width/height/factor are declared IValue on the node, read as Value)
NodeResult node() {
    return make_node({{"width", {std::nullopt, SocketType::IValue}},
                      {"height", {std::nullopt, SocketType::IValue}},
                      {"left", {std::nullopt, SocketType::IColor}},
                      {"right", {std::nullopt, SocketType::IColor}},
                      {"factor", {std::nullopt, SocketType::IValue}}},
                     {{"color", SocketValue(SocketType::IColor)}},
                     [](const Sockets& inputs, Sockets& outputs) -> ShaderResult {
                         Args a{inputs};
                         const SocketValue* width = a.get("width", SocketType::Value);
                         const SocketValue* height = a.get("height", SocketType::Value);
                         const SocketValue* left = a.get("left", SocketType::IColor);
                         const SocketValue* right = a.get("right", SocketType::IColor);
                         const SocketValue* factor = a.get("factor", SocketType::Value);
                         if (a.failed) return a.err;
                         ShaderError e;
                         SocketValue* out = get_output(outputs, "color", SocketType::IColor, &e);
                         if (!out) return e;
                         a.need("width", width);
                         a.need("height", height);
                         a.need("left", left);
                         a.need("right", right);
                         if (ShaderResult m = a.missing_error()) return m;
                         const float f = factor->as_value().value_or(DEFAULT_FACTOR);
                         DeviceImage<Color> res(sat_u32(*width->as_value()), sat_u32(*height->as_value()));
                         Device& d = Device::current();
                         d.check(eray_node_mix_color(d.ctx(), res.width, res.height, left->as_icolor()->view(),
                                                     right->as_icolor()->view(), f,
                                                     reinterpret_cast<float*>(res.data())));
                         out->as_icolor() = res;
                         return std::nullopt;
                     });
}

Status graph(GraphResult* out) {  // mix_color.rs:28-54
    GraphResult g;
    g.inputs = {{"width", SocketValue(SocketType::IValue)},
                {"height", SocketValue(SocketType::IValue)},
                {"left", SocketValue(SocketType::IColor)},
                {"right", SocketValue(SocketType::IColor)},
                {"factor", SocketValue::value(DEFAULT_FACTOR)}};
    NodeResult n = node();
    if (Status s = connect(n, {{"width", ssref_graph("width")},
                               {"height", ssref_graph("height")},
                               {"left", ssref_graph("left")},
                               {"right", ssref_graph("right")},
                               {"factor", ssref_graph("factor")}}))
        return s;
    g.nodes["mix"] = std::move(n);
    g.outputs["color"] = {ssref_node("mix", "color"), SocketValue(SocketType::IColor)};
    *out = std::move(g);
    return std::nullopt;
}
}  // namespace mix_color

std::vector<ImportedNode<Unvalidated>> elib() {  // shaderlib/mod.rs:19-40
    std::vector<ImportedNode<Unvalidated>> lib;
    GraphResult g;
    if (!flat_color::graph(&g)) lib.emplace_back("flat_color", g);
    if (!wave::graph(&g)) lib.emplace_back("wave", g);
    if (!rgb::graph(&g)) lib.emplace_back("rgb", g);
    if (!mix_color::graph(&g)) lib.emplace_back("mix_color", g);
    return lib;
}

Status example_material(Material* out) {  // main.rs:80-144
    GraphResult g;
    g.inputs = {{"width", SocketValue(SocketType::Value)},
                {"height", SocketValue(SocketType::Value)},
                {"x_fac", SocketValue::value(wave::DEFAULT_FACTOR)},
                {"y_fac", SocketValue::value(wave::DEFAULT_FACTOR)},
                {"red", SocketValue::value(1.0f)},
                {"green", SocketValue::value(1.0f)},
                {"blue", SocketValue::value(1.0f)},
                {"factor", SocketValue::value(0.5f)}};
    GraphResult sub;
    if (Status s = wave::graph(&sub)) return s;
    Node<Unvalidated> wave_node(ImportedNode<Unvalidated>("wave", sub));
    if (Status s = connect(wave_node, {{"width", ssref_graph("width")},
                                       {"height", ssref_graph("height")},
                                       {"x_fac", ssref_graph("x_fac")},
                                       {"y_fac", ssref_graph("y_fac")}}))
        return s;
    if (Status s = rgb::graph(&sub)) return s;
    Node<Unvalidated> to_color(ImportedNode<Unvalidated>("rgb", sub));
    if (Status s = connect(to_color, {{"width", ssref_graph("width")},
                                      {"height", ssref_graph("height")},
                                      {"red", ssref_node("wave", "value")},
                                      {"green", ssref_node("wave", "value")},
                                      {"blue", ssref_node("wave", "value")}}))
        return s;
    if (Status s = flat_color::graph(&sub)) return s;
    Node<Unvalidated> flat(ImportedNode<Unvalidated>("flat_color", sub));
    if (Status s = connect(flat, {{"width", ssref_graph("width")},
                                  {"height", ssref_graph("height")},
                                  {"red", ssref_graph("red")},
                                  {"green", ssref_graph("green")},
                                  {"blue", ssref_graph("blue")}}))
        return s;
    if (Status s = mix_color::graph(&sub)) return s;
    Node<Unvalidated> mixer(ImportedNode<Unvalidated>("mixer", sub));
    if (Status s = connect(mixer, {{"width", ssref_graph("width")},
                                   {"height", ssref_graph("height")},
                                   {"left", ssref_node("wave_to_color", "color")},
                                   {"right", ssref_node("flat_color", "color")},
                                   {"factor", ssref_graph("factor")}}))
        return s;
    g.nodes["wave"] = std::move(wave_node);
    g.nodes["wave_to_color"] = std::move(to_color);
    g.nodes["flat_color"] = std::move(flat);
    g.nodes["mixer"] = std::move(mixer);
    g.outputs["color"] = {ssref_node("mixer", "color"), SocketValue(SocketType::IColor)};
    g.outputs["diffuse"] = {ssref_node("wave", "value"), SocketValue(SocketType::IValue)};
    Graph<Validated> v;
    if (Status s = validate(g, &v)) return s;
    *out = Material(std::move(v), {{StandardMaterialOutput::Color, "color"}, {StandardMaterialOutput::Diffuse, "diffuse"}});
    return std::nullopt;
}

}  // namespace shaderlib
}  // namespace eray
