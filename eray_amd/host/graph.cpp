// graph.cpp — shader graph of the C++ host (src/lib/shader/graph.rs, shader.rs).
#include "eray/graph.hpp"

#include <algorithm>
#include <deque>

namespace eray {
namespace shader {

const char* to_string(SocketType t) {
    switch (t) {
        case SocketType::Value: return "Value";
        case SocketType::IValue: return "IValue";
        case SocketType::Vec2: return "Vec2";
        case SocketType::IVec2: return "IVec2";
        case SocketType::Vec3: return "Vec3";
        case SocketType::IVec3: return "IVec3";
        case SocketType::Color: return "Color";
        case SocketType::IColor: return "IColor";
    }
    return "?";
}

// ------------------------------------------------------------------------- SocketValue -----
SocketValue SocketValue::value(std::optional<float> v) {
    SocketValue s(SocketType::Value);
    s.value_ = v;
    return s;
}
SocketValue SocketValue::vec2(std::optional<std::array<float, 2>> v) {
    SocketValue s(SocketType::Vec2);
    s.vec2_ = v;
    return s;
}
SocketValue SocketValue::vec3(std::optional<std::array<float, 3>> v) {
    SocketValue s(SocketType::Vec3);
    s.vec3_ = v;
    return s;
}
SocketValue SocketValue::color(std::optional<eray::Color> v) {
    SocketValue s(SocketType::Color);
    s.color_ = v;
    return s;
}
SocketValue SocketValue::ivalue(std::optional<DeviceImage<float>> v) {
    SocketValue s(SocketType::IValue);
    s.ivalue_ = std::move(v);
    return s;
}
SocketValue SocketValue::icolor(std::optional<DeviceImage<eray::Color>> v) {
    SocketValue s(SocketType::IColor);
    s.icolor_ = std::move(v);
    return s;
}

bool SocketValue::is_none() const {
    switch (type_) {
        case SocketType::Value: return !value_;
        case SocketType::Vec2: return !vec2_;
        case SocketType::Vec3: return !vec3_;
        case SocketType::Color: return !color_;
        case SocketType::IValue: return !ivalue_;
        case SocketType::IColor: return !icolor_;
        case SocketType::IVec2:
        case SocketType::IVec3: return true;  // vector images do not reach this path
    }
    return true;
}

void SocketValue::set_default() {  // graph.rs:66-74: the kind's default, images empty
    switch (type_) {
        case SocketType::Value: value_ = 0.0f; break;
        case SocketType::Vec2: vec2_ = std::array<float, 2>{0.0f, 0.0f}; break;
        case SocketType::Vec3: vec3_ = std::array<float, 3>{0.0f, 0.0f, 0.0f}; break;
        case SocketType::Color: color_ = eray::Color(); break;
        case SocketType::IValue: ivalue_ = DeviceImage<float>(); break;
        case SocketType::IColor: icolor_ = DeviceImage<eray::Color>(); break;
        default: break;
    }
}

bool SocketValue::operator==(const SocketValue& o) const {
    return type_ == o.type_ && value_ == o.value_ && vec2_ == o.vec2_ && vec3_ == o.vec3_ &&
           color_ == o.color_ && ivalue_ == o.ivalue_ && icolor_ == o.icolor_;
}

// ------------------------------------------------------------------------------ errors -----
namespace {
std::string side_name(Side s) { return s == Side::Input ? "Input" : "Output"; }
std::string join(const std::vector<Name>& v) {
    std::string r;
    for (size_t i = 0; i < v.size(); ++i) r += (i ? ", " : "") + v[i];
    return r;
}
}  // namespace

std::string ShaderError::to_string() const {  // shader.rs:10-41 messages
    switch (kind) {
        case Kind::Missing:
        case Kind::MissingMany: return "Missing " + join(names) + " on " + side_name(side) + " side";
        case Kind::MismatchedTypes:
            return "Mismatched type between " + (names.size() > 0 ? names[0] : "") + " and " +
                   (names.size() > 1 ? names[1] : "");
        case Kind::InvalidType:
            return std::string("Invalid type ") + shader::to_string(got) + " for " + (names.empty() ? "" : names[0]) +
                   ", expected " + shader::to_string(expected);
        case Kind::Unknown: return "Unknown error" + (message.empty() ? "" : ": " + message);
    }
    return "?";
}

bool ShaderError::operator==(const ShaderError& o) const {
    return kind == o.kind && side == o.side && names == o.names && got == o.got && expected == o.expected &&
           message == o.message;
}

std::string GraphError::to_string() const {  // graph.rs:321-347 messages
    switch (kind) {
        case Kind::UnlinkedUnsetGraphOutput: return "Graph output `" + name + "` left unlinked";
        case Kind::Cycle: {
            std::string p;
            for (size_t i = 0; i < during.size(); ++i) p += (i ? ", " : "") + during[i];
            return "Detected a cycle while validating the path [" + p + "]; cycle is from a `" + source_socket +
                   "` socket to a `" + target_socket + "` socket, reaching node `" + detected + "`";
        }
        case Kind::Shader: return "A shader function returned an error: " + shader.to_string();
        case Kind::Missing: return "Referencing missing " + side_name(side) + " socket " + name;
    }
    return "?";
}

bool GraphError::operator==(const GraphError& o) const {
    return kind == o.kind && name == o.name && side == o.side && during == o.during &&
           source_socket == o.source_socket && target_socket == o.target_socket && detected == o.detected &&
           shader == o.shader;
}

// get_sv! (shader.rs:140-177)
const SocketValue* get_input(const Sockets& inputs, const Name& name, SocketType kind, ShaderError* err) {
    auto it = inputs.find(name);
    if (it == inputs.end()) {
        *err = ShaderError{ShaderError::Kind::Missing, Side::Input, {name}};
        return nullptr;
    }
    if (it->second.type() != kind) {
        *err = ShaderError{ShaderError::Kind::InvalidType, Side::Input, {name}, it->second.type(), kind};
        return nullptr;
    }
    return &it->second;
}

SocketValue* get_output(Sockets& outputs, const Name& name, SocketType kind, ShaderError* err) {
    auto it = outputs.find(name);
    if (it == outputs.end()) {
        *err = ShaderError{ShaderError::Kind::Missing, Side::Output, {name}};
        return nullptr;
    }
    if (it->second.type() != kind) {
        *err = ShaderError{ShaderError::Kind::InvalidType, Side::Output, {name}, it->second.type(), kind};
        return nullptr;
    }
    return &it->second;
}

// ------------------------------------------------------------------------------- nodes -----
template <class State>
ImportedNode<State>::ImportedNode(Name n, const Graph<State>& g)
    : name(std::move(n)), inner(std::make_shared<Graph<State>>(g)) {
    for (const auto& [k, v] : g.inputs) inputs[k] = {std::nullopt, v.type()};  // graph.rs:673-685
}

template <class State>
ImportedNode<State>::ImportedNode(const ImportedNode& o)
    : name(o.name), inputs(o.inputs), inner(o.inner ? std::make_shared<Graph<State>>(*o.inner) : nullptr) {}

template <class State>
ImportedNode<State>& ImportedNode<State>::operator=(const ImportedNode& o) {
    if (this != &o) {
        name = o.name;
        inputs = o.inputs;
        inner = o.inner ? std::make_shared<Graph<State>>(*o.inner) : nullptr;
    }
    return *this;
}

template <class State>
bool ImportedNode<State>::operator==(const ImportedNode& o) const {
    return name == o.name && inputs == o.inputs && ((!inner && !o.inner) || (inner && o.inner && *inner == *o.inner));
}

template <class State>
const NodeInputs& Node<State>::inputs() const {
    return v.index() == 0 ? std::get<0>(v).inputs : std::get<1>(v).inputs;
}

template <class State>
std::map<Name, const SocketValue*> Node<State>::outputs() const {
    std::map<Name, const SocketValue*> r;
    if (v.index() == 0) {
        for (const auto& [k, val] : std::get<0>(v).outputs) r[k] = &val;
    } else {
        for (const auto& [k, val] : std::get<1>(v).inner->outputs) r[k] = &val.second;
    }
    return r;
}

template <class State>
Status Node<State>::set_input(const Name& name, std::optional<SocketRef> socket_ref) {
    NodeInputs& in = v.index() == 0 ? std::get<0>(v).inputs : std::get<1>(v).inputs;
    auto it = in.find(name);
    if (it == in.end()) {
        GraphError e;
        e.kind = GraphError::Kind::Missing;
        e.side = Side::Input;
        e.name = name;
        return e;
    }
    it->second.first = std::move(socket_ref);
    return std::nullopt;
}

template struct ImportedNode<Unvalidated>;
template struct ImportedNode<Validated>;
template struct Node<Unvalidated>;
template struct Node<Validated>;

// ---------------------------------------------------------------------------- validate -----
namespace {
bool contains(const std::vector<NodeId>& v, const NodeId& x) { return std::find(v.begin(), v.end(), x) != v.end(); }
}  // namespace

Status validate(const Graph<Unvalidated>& g, Graph<Validated>* out) {
    std::vector<NodeId> path, visited;
    std::deque<NodeId> next;
    for (const auto& [output, entry] : g.outputs) {
        const auto& [socket_ref, value] = entry;
        if (!socket_ref) {  // an output must be linked or already hold a value
            if (value.is_none()) {
                GraphError e;
                e.kind = GraphError::Kind::UnlinkedUnsetGraphOutput;
                e.name = output;
                return e;
            }
            continue;
        }
        if (socket_ref->kind != SocketRef::Kind::Node) continue;
        if (contains(visited, socket_ref->node)) continue;
        next.push_back(socket_ref->node);
        while (!next.empty()) {  // depth-first through push_front (graph.rs:444-485)
            const NodeId current = next.front();
            next.pop_front();
            auto it = g.nodes.find(current);
            if (it == g.nodes.end()) continue;
            visited.push_back(current);
            path.push_back(current);
            bool pushed_some = false;
            for (const auto& [input, inp] : it->second.inputs()) {
                const auto& sref = inp.first;
                if (!sref || sref->kind != SocketRef::Kind::Node) continue;
                if (contains(path, sref->node)) {
                    GraphError e;
                    e.kind = GraphError::Kind::Cycle;
                    e.detected = sref->node;
                    e.target_socket = sref->socket;
                    e.source_socket = input;
                    e.during = path;
                    return e;
                }
                if (contains(visited, sref->node)) continue;
                next.push_front(sref->node);
                pushed_some = true;
            }
            if (!pushed_some) path.pop_back();
        }
    }
    Graph<Validated> r;
    r.inputs = g.inputs;
    r.outputs = g.outputs;
    for (const auto& [id, node] : g.nodes) {
        if (!node.is_imported()) {
            r.nodes[id] = Node<Validated>(std::get<0>(node.v));
        } else {
            const ImportedNode<Unvalidated>& im = std::get<1>(node.v);
            ImportedNode<Validated> vn;
            vn.name = im.name;
            vn.inputs = im.inputs;
            vn.inner = std::make_shared<Graph<Validated>>();
            if (Status s = validate(*im.inner, vn.inner.get())) return s;
            r.nodes[id] = Node<Validated>(std::move(vn));
        }
    }
    *out = std::move(r);
    return std::nullopt;
}

// --------------------------------------------------------------------------------- run -----
namespace {
[[noreturn]] void panic(const std::string& what) { throw Failure(ERAY_E_MISSING, what); }

const SocketValue& node_output(Graph<Validated>& g, const NodeId& id, const Name& field) {
    auto it = g.nodes.find(id);
    if (it == g.nodes.end()) panic("node `" + id + "` not found");
    const auto outs = it->second.outputs();
    auto o = outs.find(field);
    if (o == outs.end()) panic("Output `" + field + "` not found for node `" + id + "`.");
    return *o->second;
}

const SocketValue& graph_input(Graph<Validated>& g, const Name& field) {
    auto it = g.inputs.find(field);
    if (it == g.inputs.end()) panic("graph input `" + field + "` not found");
    return it->second;
}

Status run_node(Graph<Validated>& g, const NodeId& node_id) {
    auto it = g.nodes.find(node_id);
    if (it == g.nodes.end()) panic("node `" + node_id + "` not found");
    {  // skip a node whose outputs are all computed (graph.rs:545-553)
        bool all = true;
        for (const auto& [k, v] : it->second.outputs()) all = all && !v->is_none();
        if (all) return std::nullopt;
    }
    const Node<Validated> cur = it->second;  // the reference clones the node (graph.rs:555)
    auto value_of = [&](const SocketRef& sref, Status* st) -> SocketValue {
        if (sref.kind == SocketRef::Kind::Node) {
            if ((*st = run_node(g, sref.node))) return SocketValue();
            return node_output(g, sref.node, sref.socket);
        }
        return graph_input(g, sref.socket);
    };
    if (!cur.is_imported()) {
        Sockets inputs;
        for (const auto& [name, inp] : std::get<0>(cur.v).inputs) {
            if (inp.first) {
                Status st;
                SocketValue v = value_of(*inp.first, &st);
                if (st) return st;
                inputs[name] = std::move(v);
            } else {
                inputs[name] = SocketValue(inp.second);  // r#type.into(): the kind, None
            }
        }
        GraphNode& node = g.nodes[node_id].graph_node();
        if (ShaderResult r = node.shader.call(inputs, node.outputs)) {
            GraphError e;
            e.kind = GraphError::Kind::Shader;
            e.shader = *r;
            return e;
        }
    } else {
        for (const auto& [name, inp] : std::get<1>(cur.v).inputs) {
            if (inp.first) {
                Status st;
                SocketValue v = value_of(*inp.first, &st);
                if (st) return st;
                g.nodes[node_id].imported().inner->inputs[name] = std::move(v);
            } else {
                auto& inner_inputs = g.nodes[node_id].imported().inner->inputs;
                auto f = inner_inputs.find(name);
                if (f == inner_inputs.end()) panic("imported input `" + name + "` not found");
                f->second.set_default();
            }
        }
        if (Status st = run(*g.nodes[node_id].imported().inner)) return st;
    }
    return std::nullopt;
}
}  // namespace

Status run(Graph<Validated>& g) {
    std::map<Name, std::pair<std::optional<SocketRef>, SocketValue>> outputs;
    for (const auto& [name, entry] : g.outputs) {
        auto [socket_ref, value] = entry;
        if (!value.is_none()) continue;  // outputs that already hold a value are dropped
        if (!socket_ref) {
            value.set_default();
        } else if (socket_ref->kind == SocketRef::Kind::Node) {
            if (Status st = run_node(g, socket_ref->node)) return st;
            value = node_output(g, socket_ref->node, socket_ref->socket);
        } else {
            value = graph_input(g, socket_ref->socket);
        }
        outputs[name] = {socket_ref, value};
    }
    g.outputs = std::move(outputs);
    return std::nullopt;
}

}  // namespace shader
}  // namespace eray
