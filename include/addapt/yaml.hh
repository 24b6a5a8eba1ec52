// Minimal YAML subset for addapt config files (no anchors, tags or
// multi-document streams).  Parse errors throw std::string "YAML: ...".
#pragma once

#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace addapt {
namespace yaml {

struct Node {
    enum Kind { NONE, SCALAR, MAP, LIST } kind = NONE;
    std::string scalar;
    std::vector<std::pair<std::string, Node>> map;   // in file order
    std::vector<Node> list;

    explicit operator bool() const { return kind != NONE; }
    const Node &operator[](const std::string &key) const;   // NONE node if absent
    const Node &operator[](size_t i) const;
    std::string as_string() const;   // throws unless SCALAR
};

Node parse(const std::string &text);
Node load_file(const std::string &path);

}  // namespace yaml
}  // namespace addapt
