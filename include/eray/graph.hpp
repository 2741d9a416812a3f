// graph.hpp — the shader graph of the C++ host: sockets, Shader, GraphNode / ImportedNode,
// Graph<Unvalidated> -> validate() -> Graph<Validated> -> run().  Mirrors the reference's
// src/lib/shader/graph.rs and shader.rs (same names, socket semantics and errors); the node
// operators of shaderlib.hpp evaluate on the GPU through the C-ABI.
//
// Rust -> C++: HashMap -> std::map (deterministic order), Option -> std::optional,
// Result<_, Error> -> an Error value that is empty on success (`ok()`), the typestate
// Graph<Unvalidated> / Graph<Validated> -> Graph<State> with the same two tag types.
#pragma once

#include <array>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <utility>
#include <variant>
#include <vector>

#include "image.hpp"

namespace eray {
namespace shader {

using Name = std::string;    // graph.rs:229 Name(String)
using NodeId = std::string;  // graph.rs:210 NodeId(String)

// graph.rs:160-169 (socket_value!): a scalar kind and its image kind
enum class SocketType { Value, IValue, Vec2, IVec2, Vec3, IVec3, Color, IColor };
const char* to_string(SocketType t);

// graph.rs:26-83 SocketValue: one Option per kind; images live on the device (IValue, IColor).
class SocketValue {
public:
    SocketValue() : SocketValue(SocketType::Value) {}
    SocketValue(SocketType t) : type_(t) {}  // From<SocketType>: the kind with None
    static SocketValue value(std::optional<float> v);
    static SocketValue vec2(std::optional<std::array<float, 2>> v);
    static SocketValue vec3(std::optional<std::array<float, 3>> v);
    static SocketValue color(std::optional<eray::Color> v);
    static SocketValue ivalue(std::optional<DeviceImage<float>> v);
    static SocketValue icolor(std::optional<DeviceImage<eray::Color>> v);

    SocketType type() const { return type_; }  // From<&SocketValue> for SocketType
    bool is_none() const;                        // graph.rs:56-64
    void set_default();                          // graph.rs:66-74 (images: an empty image)

    std::optional<float>& as_value() { return value_; }
    const std::optional<float>& as_value() const { return value_; }
    std::optional<std::array<float, 2>>& as_vec2() { return vec2_; }
    std::optional<std::array<float, 3>>& as_vec3() { return vec3_; }
    std::optional<eray::Color>& as_color() { return color_; }
    std::optional<DeviceImage<float>>& as_ivalue() { return ivalue_; }
    const std::optional<DeviceImage<float>>& as_ivalue() const { return ivalue_; }
    std::optional<DeviceImage<eray::Color>>& as_icolor() { return icolor_; }
    const std::optional<DeviceImage<eray::Color>>& as_icolor() const { return icolor_; }

    bool operator==(const SocketValue& o) const;
    bool operator!=(const SocketValue& o) const { return !(*this == o); }

private:
    SocketType type_;
    std::optional<float> value_;
    std::optional<std::array<float, 2>> vec2_;
    std::optional<std::array<float, 3>> vec3_;
    std::optional<eray::Color> color_;
    std::optional<DeviceImage<float>> ivalue_;
    std::optional<DeviceImage<eray::Color>> icolor_;
};

// graph.rs:246-253: a node output or a graph input
struct SocketRef {
    enum class Kind { Node, Graph } kind = Kind::Graph;
    NodeId node;
    Name socket;
    static SocketRef graph(Name socket) { return SocketRef{Kind::Graph, {}, std::move(socket)}; }
    static SocketRef of_node(NodeId node, Name socket) { return SocketRef{Kind::Node, std::move(node), std::move(socket)}; }
    bool operator==(const SocketRef& o) const { return kind == o.kind && node == o.node && socket == o.socket; }
};
// sref! / ssref! (graph.rs:255-300)
inline std::optional<SocketRef> ssref_graph(Name socket) { return SocketRef::graph(std::move(socket)); }
inline std::optional<SocketRef> ssref_node(NodeId node, Name socket) {
    return SocketRef::of_node(std::move(node), std::move(socket));
}

enum class Side { Input, Output };  // shader.rs:44-50

// shader.rs:8-41 shader::Error
struct ShaderError {
    enum class Kind { Missing, MissingMany, MismatchedTypes, InvalidType, Unknown } kind = Kind::Unknown;
    Side side = Side::Input;
    std::vector<Name> names;  // Missing: 1, MissingMany: n, MismatchedTypes / InvalidType: 1-2
    SocketType got = SocketType::Value, expected = SocketType::Value;
    std::string message;  // Unknown
    std::string to_string() const;
    bool operator==(const ShaderError& o) const;
};

using Sockets = std::map<Name, SocketValue>;
using ShaderResult = std::optional<ShaderError>;  // Ok(()) = nullopt

// shader.rs:52-100: a node's function over its inputs and outputs
class Shader {
public:
    using Fn = std::function<ShaderResult(const Sockets& inputs, Sockets& outputs)>;
    Shader() : fn_([](const Sockets&, Sockets&) { return ShaderResult{}; }) {}  // Default: no-op
    explicit Shader(Fn fn) : fn_(std::move(fn)) {}
    ShaderResult call(const Sockets& inputs, Sockets& outputs) const { return fn_(inputs, outputs); }

private:
    Fn fn_;
};

// get_sv! (shader.rs:140-177): the named input/output as its kind, or Missing / InvalidType
const SocketValue* get_input(const Sockets& inputs, const Name& name, SocketType kind, ShaderError* err);
SocketValue* get_output(Sockets& outputs, const Name& name, SocketType kind, ShaderError* err);

// graph.rs:319-347 graph::Error
struct GraphError {
    enum class Kind { UnlinkedUnsetGraphOutput, Cycle, Shader, Missing } kind = Kind::Shader;
    Name name;                      // UnlinkedUnsetGraphOutput, Missing
    Side side = Side::Input;        // Missing
    std::vector<NodeId> during;     // Cycle
    Name source_socket, target_socket;
    NodeId detected;
    ShaderError shader;             // Shader
    std::string to_string() const;
    bool operator==(const GraphError& o) const;
};
using Status = std::optional<GraphError>;  // Ok(()) = nullopt

struct Unvalidated {};  // graph.rs:313-318
struct Validated {};

template <class State>
struct Graph;

using NodeInputs = std::map<Name, std::pair<std::optional<SocketRef>, SocketType>>;

// graph.rs:611-621: a node with its own Shader
struct GraphNode {
    NodeInputs inputs;
    Sockets outputs;
    Shader shader;
    bool operator==(const GraphNode& o) const { return inputs == o.inputs && outputs == o.outputs; }  // ignores shader
};

// graph.rs:639-701: a sub-graph used as a node
template <class State>
struct ImportedNode {
    Name name;
    NodeInputs inputs;
    std::shared_ptr<Graph<State>> inner;  // deep-copied with the node (value semantics)

    ImportedNode() = default;
    ImportedNode(Name n, const Graph<State>& g);  // From<(T, Graph<State>)>
    ImportedNode(const ImportedNode& o);
    ImportedNode& operator=(const ImportedNode& o);
    ImportedNode(ImportedNode&&) = default;
    ImportedNode& operator=(ImportedNode&&) = default;
    bool operator==(const ImportedNode& o) const;
};

// graph.rs:703-800: a node is a GraphNode or an ImportedNode
template <class State>
struct Node {
    std::variant<GraphNode, ImportedNode<State>> v;

    Node() : v(GraphNode{}) {}
    Node(GraphNode n) : v(std::move(n)) {}
    Node(ImportedNode<State> n) : v(std::move(n)) {}
    bool is_imported() const { return v.index() == 1; }
    GraphNode& graph_node() { return std::get<0>(v); }
    ImportedNode<State>& imported() { return std::get<1>(v); }
    const NodeInputs& inputs() const;
    std::map<Name, const SocketValue*> outputs() const;
    // graph.rs:727-746 (Node<Unvalidated>::set_input): Missing(Input, name) if absent
    Status set_input(const Name& name, std::optional<SocketRef> socket_ref);
    bool operator==(const Node& o) const { return v == o.v; }
};

// graph.rs:355-367
template <class State>
struct Graph {
    Sockets inputs;
    std::map<Name, std::pair<std::optional<SocketRef>, SocketValue>> outputs;
    std::map<NodeId, Node<State>> nodes;
    bool operator==(const Graph& o) const { return inputs == o.inputs && outputs == o.outputs && nodes == o.nodes; }
};

// graph.rs:408-493 Graph<Unvalidated>::validate: cycle detection from every graph output
// (depth-first, the reference's path/visited bookkeeping and error fields).
Status validate(const Graph<Unvalidated>& graph, Graph<Validated>* out);

// graph.rs:496-609 Graph<Validated>::run / run_node: pull evaluation from the graph outputs.
// Outputs that already hold a value are dropped, as the reference's run does (graph.rs:505).
Status run(Graph<Validated>& graph);

}  // namespace shader
}  // namespace eray
