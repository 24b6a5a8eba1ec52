// Minimal YAML subset reader for addapt config files (include/addapt/yaml.hh).
#include "addapt/yaml.hh"

#include <fstream>
#include <sstream>

namespace addapt {
namespace yaml {

namespace {

const Node &none() {
    static const Node n;
    return n;
}

struct Line {
    int indent;
    std::string text;   // without indent and comment
    int no;
};

std::string strip_comment(const std::string &s) {
    bool sq = false, dq = false;
    for (size_t k = 0; k < s.size(); k++) {
        const char c = s[k];
        if (c == '\'' && !dq) sq = !sq;
        else if (c == '"' && !sq) dq = !dq;
        else if (c == '#' && !sq && !dq && (k == 0 || s[k - 1] == ' ' || s[k - 1] == '\t')) return s.substr(0, k);
    }
    return s;
}

std::string trim(const std::string &s) {
    size_t a = s.find_first_not_of(" \t\r"), b = s.find_last_not_of(" \t\r");
    return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

[[noreturn]] void fail(int no, const std::string &msg) {
    throw std::string("YAML: line " + std::to_string(no) + ": " + msg);
}

std::string unquote(const std::string &s, int no) {
    if (s.size() >= 2 && (s[0] == '"' || s[0] == '\'')) {
        if (s.back() != s[0]) fail(no, "unterminated quoted scalar");
        std::string out;
        for (size_t k = 1; k + 1 < s.size(); k++) {
            if (s[0] == '"' && s[k] == '\\' && k + 2 < s.size()) {
                const char e = s[++k];
                out += e == 'n' ? '\n' : e == 't' ? '\t' : e;
            } else if (s[0] == '\'' && s[k] == '\'' && k + 2 < s.size() && s[k + 1] == '\'') {
                out += '\'';
                k++;
            } else {
                out += s[k];
            }
        }
        return out;
    }
    return s;
}

// split "a, 'b, c', d" at top-level commas
std::vector<std::string> split_flow(const std::string &s, int no) {
    std::vector<std::string> out;
    std::string cur;
    bool sq = false, dq = false;
    for (char c : s) {
        if (c == '\'' && !dq) sq = !sq;
        if (c == '"' && !sq) dq = !dq;
        if (c == ',' && !sq && !dq) {
            out.push_back(trim(cur));
            cur.clear();
        } else {
            cur += c;
        }
    }
    if (sq || dq) fail(no, "unterminated quote in flow sequence");
    if (!trim(cur).empty() || !out.empty()) out.push_back(trim(cur));
    return out;
}

Node scalar_or_flow(const std::string &v, int no) {
    Node n;
    if (!v.empty() && v[0] == '[') {
        if (v.back() != ']') fail(no, "unterminated flow sequence");
        n.kind = Node::LIST;
        for (auto &item : split_flow(v.substr(1, v.size() - 2), no)) {
            Node c;
            c.kind = Node::SCALAR;
            c.scalar = unquote(item, no);
            n.list.push_back(c);
        }
        return n;
    }
    if (!v.empty() && v[0] == '{') fail(no, "flow mappings are not supported");
    n.kind = Node::SCALAR;
    n.scalar = unquote(v, no);
    return n;
}

// key: value split at the first ': ' (or trailing ':') outside quotes
bool split_key(const std::string &t, std::string &key, std::string &val) {
    bool sq = false, dq = false;
    for (size_t k = 0; k < t.size(); k++) {
        const char c = t[k];
        if (c == '\'' && !dq) sq = !sq;
        else if (c == '"' && !sq) dq = !dq;
        else if (c == ':' && !sq && !dq && (k + 1 == t.size() || t[k + 1] == ' ' || t[k + 1] == '\t')) {
            key = trim(t.substr(0, k));
            val = trim(t.substr(k + 1));
            return true;
        }
    }
    return false;
}

Node parse_block(const std::vector<Line> &ls, size_t &k, int indent);

Node parse_value(const std::vector<Line> &ls, size_t &k, int parent_indent, const std::string &inline_val, int no) {
    if (!inline_val.empty()) return scalar_or_flow(inline_val, no);
    if (k < ls.size() && ls[k].indent > parent_indent) return parse_block(ls, k, ls[k].indent);
    // a list may sit at the parent's indentation under a key ("key:\n- a")
    if (k < ls.size() && ls[k].indent == parent_indent && ls[k].text.rfind("- ", 0) == 0)
        return parse_block(ls, k, parent_indent);
    Node n;
    n.kind = Node::SCALAR;   // "key:" with nothing = empty scalar (YAML null)
    return n;
}

Node parse_block(const std::vector<Line> &ls, size_t &k, int indent) {
    Node n;
    const bool is_list = ls[k].text == "-" || ls[k].text.rfind("- ", 0) == 0;
    n.kind = is_list ? Node::LIST : Node::MAP;
    while (k < ls.size() && ls[k].indent == indent) {
        const Line &l = ls[k];
        if (is_list) {
            if (!(l.text == "-" || l.text.rfind("- ", 0) == 0)) fail(l.no, "expected a '- ' list item");
            const std::string rest = trim(l.text.substr(1));
            k++;
            std::string key, val;
            if (!rest.empty() && split_key(rest, key, val)) fail(l.no, "mappings inside list items are not supported");
            n.list.push_back(parse_value(ls, k, indent, rest, l.no));
        } else {
            std::string key, val;
            if (!split_key(l.text, key, val)) fail(l.no, "expected 'key: value'");
            key = unquote(key, l.no);
            for (auto &kv : n.map)
                if (kv.first == key) fail(l.no, "duplicate key '" + key + "'");
            k++;
            n.map.emplace_back(key, parse_value(ls, k, indent, val, l.no));
        }
    }
    if (k < ls.size() && ls[k].indent > indent) fail(ls[k].no, "unexpected indentation");
    return n;
}

}  // namespace

const Node &Node::operator[](const std::string &key) const {
    if (kind != MAP) return none();
    for (auto &kv : map)
        if (kv.first == key) return kv.second;
    return none();
}

const Node &Node::operator[](size_t i) const {
    if (kind != LIST || i >= list.size()) return none();
    return list[i];
}

std::string Node::as_string() const {
    if (kind != SCALAR) throw std::string("YAML: expected a scalar");
    return scalar;
}

Node parse(const std::string &text) {
    std::vector<Line> ls;
    std::istringstream in(text);
    std::string raw;
    int no = 0;
    while (std::getline(in, raw)) {
        no++;
        if (raw.find('\t') != std::string::npos && raw.find_first_not_of(" \t") != std::string::npos &&
            raw.find('\t') < raw.find_first_not_of(" \t"))
            fail(no, "tab indentation");
        const std::string s = strip_comment(raw);
        const std::string t = trim(s);
        if (t.empty() || t == "---" || t == "...") continue;
        ls.push_back(Line{int(s.find_first_not_of(' ')), t, no});
    }
    if (ls.empty()) return Node{};
    size_t k = 0;
    Node n = parse_block(ls, k, ls[0].indent);
    if (k != ls.size()) fail(ls[k].no, "unexpected content");
    return n;
}

Node load_file(const std::string &path) {
    std::ifstream f(path);
    if (!f) throw std::string("YAML: bad file: " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse(ss.str());
}

}  // namespace yaml
}  // namespace addapt
