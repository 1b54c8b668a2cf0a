// Native streaming GEXF scanner for the loader of DPathSim_APVPA.py:114-129
// (read_dblp_nx_file -> networkx.read_gexf, :116; vertex tuples :120-121,
// edge tuples :123-124).  Host code, no HIP.
//
// It does the per-element work of dpathsim/gexf.py's iterparse loop -- node
// order by first appearance, in-place updates of repeated node ids, the
// node_type attvalue, edge endpoints interned to node indices, the relationship
// (attvalue titled "label", overridden by the XML label attribute), edge ids as
// multigraph keys, "mutual" edges doubled -- over an mmap'ed file, and hands
// back flat arrays; gexf.py applies the (vectorised) networkx key-collapse and
// adjacency ordering to them exactly as it does for its own loop.
//
// Anything outside that subset returns status 1 and the caller runs
// the Python parser, which raises the reference's exceptions: nested <nodes>,
// DOCTYPE, an attvalue without a value or with an undefined `for`, non-string
// attribute types whose values would not convert, edges whose type contradicts
// the graph's default edge type.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

#include "dps_host.hpp"

namespace {

constexpr int kOk = 0;
constexpr int kFallback = 1;

struct AttrDef {
  std::string title, type;
  bool has_type = false;
};

struct Gexf {
  bool directed = true;
  std::vector<std::string> node_ids;
  std::vector<std::string> labels;
  std::vector<uint8_t> label_null;
  std::vector<int32_t> ntype;                    // -1: no node_type (edge-only node)
  std::vector<std::string> type_names;
  std::unordered_map<std::string, int32_t> type_map;
  std::unordered_map<std::string, int32_t> node_index;
  std::vector<int32_t> e_src, e_dst, e_rel;          // rel -1: missing
  std::vector<int64_t> key_off;                      // edge id: offset into key_buf, -1: none
  std::string key_buf;                               // (ids are compared only for repeated pairs)
  std::vector<std::string> rel_names;
  std::unordered_map<std::string, int32_t> rel_map;
};

int32_t intern(std::unordered_map<std::string, int32_t>& m, std::vector<std::string>* names,
               const std::string& s) {
  auto it = m.find(s);
  if (it != m.end()) return it->second;
  const int32_t id = static_cast<int32_t>(m.size());
  m.emplace(s, id);
  if (names) names->push_back(s);
  return id;
}

void put_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

// XML attribute value -> text (entities and character references decoded,
// attribute-value whitespace normalisation of tab / newline / CR to spaces).
bool decode(std::string_view v, std::string& out) {
  out.clear();
  for (size_t i = 0; i < v.size(); ++i) {
    const char c = v[i];
    if (c == '\t' || c == '\n' || c == '\r') { out.push_back(' '); continue; }
    if (c != '&') { out.push_back(c); continue; }
    const size_t semi = v.find(';', i);
    if (semi == std::string_view::npos) return false;
    const std::string_view ent = v.substr(i + 1, semi - i - 1);
    if (ent == "amp") out.push_back('&');
    else if (ent == "lt") out.push_back('<');
    else if (ent == "gt") out.push_back('>');
    else if (ent == "quot") out.push_back('"');
    else if (ent == "apos") out.push_back('\'');
    else if (ent.size() > 1 && ent[0] == '#') {
      char* endp = nullptr;
      const std::string num(ent.substr(ent[1] == 'x' ? 2 : 1));
      const unsigned long cp = std::strtoul(num.c_str(), &endp, ent[1] == 'x' ? 16 : 10);
      if (num.empty() || *endp || cp > 0x10FFFF) return false;
      put_utf8(out, static_cast<uint32_t>(cp));
    } else {
      return false;   // undefined entity: the Python parser reports it
    }
    i = semi;
  }
  return true;
}

bool stringy(const AttrDef& d) {
  return !d.has_type || d.type == "string" || d.type == "liststring" || d.type == "anyURI";
}

// Would gexf.py's _convert accept this value for a non-string type?
bool converts(const AttrDef& d, const std::string& v) {
  if (stringy(d)) return true;
  const std::string& t = d.type;
  if (t == "integer" || t == "long" || t == "short" || t == "byte") return false;   // int(): leave to Python
  if (t == "float" || t == "double") return false;
  if (t == "boolean") return v == "true" || v == "false" || v == "True" || v == "False" ||
                             v == "1" || v == "0";
  return true;   // unknown types are kept as strings by _convert
}

struct Attr {
  std::string_view name;
  std::string_view raw;
};

const Attr* find(const std::vector<Attr>& a, std::string_view n) {
  for (const Attr& x : a)
    if (x.name == n) return &x;
  return nullptr;
}

// True unless [b, e) is an XML declaration naming an encoding other than
// UTF-8 / ASCII (those files go to the caller's parser, which decodes them).
bool utf8_declaration(const char* b, const char* e) {
  const std::string_view d(b, static_cast<size_t>(e - b));
  if (d.substr(0, 5) != "<?xml") return true;
  const size_t k = d.find("encoding");
  if (k == std::string_view::npos) return true;
  size_t i = k + 8;
  while (i < d.size() && (d[i] == ' ' || d[i] == '=' || d[i] == '\t')) ++i;
  if (i >= d.size() || (d[i] != '"' && d[i] != '\'')) return false;
  const char q = d[i++];
  const size_t j = d.find(q, i);
  if (j == std::string_view::npos) return false;
  std::string enc(d.substr(i, j - i));
  for (char& c : enc) c = static_cast<char>(c >= 'A' && c <= 'Z' ? c - 'A' + 'a' : c);
  return enc == "utf-8" || enc == "utf8" || enc == "ascii" || enc == "us-ascii";
}

class Scanner {
 public:
  Scanner(const char* b, const char* e, Gexf& g) : p_(b), e_(e), g_(g) {}

  int run() {
    // byte-order marks of UTF-16/32: not this scanner's encoding
    if (e_ - p_ >= 2 && ((p_[0] == '\xFF' && p_[1] == '\xFE') || (p_[0] == '\xFE' && p_[1] == '\xFF')))
      return kFallback;
    while (p_ < e_) {
      const char* lt = static_cast<const char*>(std::memchr(p_, '<', static_cast<size_t>(e_ - p_)));
      if (!lt) break;
      p_ = lt;
      if (e_ - p_ >= 2 && p_[1] == '?') {
        const char* q0 = p_;
        if (!skip_to("?>")) return kFallback;
        if (!utf8_declaration(q0, p_)) return kFallback;
        continue;
      }
      if (starts("<!--")) { if (!skip_to("-->")) return kFallback; continue; }
      if (starts("<![CDATA[")) { if (!skip_to("]]>")) return kFallback; continue; }
      if (e_ - p_ >= 2 && p_[1] == '!') return kFallback;   // DOCTYPE / declarations
      if (e_ - p_ >= 2 && p_[1] == '/') {
        p_ += 2;
        const std::string_view name = read_name();
        const char* gt = static_cast<const char*>(std::memchr(p_, '>', static_cast<size_t>(e_ - p_)));
        if (!gt) return kFallback;
        p_ = gt + 1;
        const int rc = on_end(local(name), nullptr);
        if (rc != kOk) return rc;
        continue;
      }
      ++p_;
      const std::string_view name = read_name();
      attrs_.clear();
      bool self_close = false;
      for (;;) {
        skip_ws();
        if (p_ >= e_) return kFallback;
        if (*p_ == '>') { ++p_; break; }
        if (*p_ == '/' && p_ + 1 < e_ && p_[1] == '>') { p_ += 2; self_close = true; break; }
        const std::string_view an = read_name();
        if (an.empty()) return kFallback;
        skip_ws();
        if (p_ >= e_ || *p_ != '=') return kFallback;
        ++p_;
        skip_ws();
        if (p_ >= e_ || (*p_ != '"' && *p_ != '\'')) return kFallback;
        const char q = *p_++;
        const char* ve = static_cast<const char*>(std::memchr(p_, q, static_cast<size_t>(e_ - p_)));
        if (!ve) return kFallback;
        attrs_.push_back({an, std::string_view(p_, static_cast<size_t>(ve - p_))});
        p_ = ve + 1;
      }
      const std::string_view ln = local(name);
      int rc = on_start(ln);
      if (rc == kOk && self_close) rc = on_end(ln, &attrs_);
      if (rc != kOk) return rc;
    }
    return depth_nodes_ == 0 ? kOk : kFallback;
  }

 private:
  bool starts(const char* s) const {
    const size_t n = std::strlen(s);
    return static_cast<size_t>(e_ - p_) >= n && std::memcmp(p_, s, n) == 0;
  }
  bool skip_to(const char* s) {
    const std::string_view hay(p_, static_cast<size_t>(e_ - p_));
    const size_t k = hay.find(s);
    if (k == std::string_view::npos) return false;
    p_ += k + std::strlen(s);
    return true;
  }
  void skip_ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  std::string_view read_name() {
    const char* b = p_;
    while (p_ < e_ && *p_ != ' ' && *p_ != '\t' && *p_ != '\n' && *p_ != '\r' && *p_ != '>' &&
           *p_ != '/' && *p_ != '=')
      ++p_;
    return std::string_view(b, static_cast<size_t>(p_ - b));
  }
  static std::string_view local(std::string_view n) {
    const size_t c = n.rfind(':');
    return c == std::string_view::npos ? n : n.substr(c + 1);
  }
  // decoded value of attribute n of the current start tag (false: absent)
  bool get(std::string_view n, std::string& out, bool* bad = nullptr) {
    const Attr* a = find(attrs_, n);
    if (!a) return false;
    if (!decode(a->raw, out) && bad) *bad = true;
    return true;
  }

  int on_start(std::string_view tag) {
    bool bad = false;
    if (tag == "graph") {
      std::string v;
      g_.directed = get("defaultedgetype", v, &bad) && v == "directed";
    } else if (tag == "attributes") {
      has_class_ = get("class", attr_class_, &bad);
    } else if (tag == "attribute") {
      pend_ = AttrDef();
      pend_has_ = get("id", pend_id_, &bad);
      get("title", pend_.title, &bad);
      pend_.has_type = get("type", pend_.type, &bad);
    } else if (tag == "nodes") {
      if (++depth_nodes_ > 1) return kFallback;   // GEXF sub-nodes: Python raises
    } else if (tag == "node") {
      kind_ = 1;
      if (!get("id", cur_id_, &bad)) return kFallback;
      cur_label_null_ = !get("label", cur_label_, &bad);
      cur_has_type_ = false;
    } else if (tag == "edge") {
      kind_ = 2;
      if (!get("source", cur_src_, &bad) || !get("target", cur_dst_, &bad)) return kFallback;
      cur_key_null_ = !get("id", cur_key_, &bad);
      cur_label_null_ = !get("label", cur_label_, &bad);
      cur_type_null_ = !get("type", cur_etype_, &bad);
      cur_att_label_ = false;
    } else if (tag == "attvalue") {
      av_attrs_ok_ = true;
      av_has_for_ = get("for", av_for_, &bad);
      av_has_value_ = get("value", av_value_, &bad);
    }
    return bad ? kFallback : kOk;
  }

  int on_end(std::string_view tag, const std::vector<Attr>*) {
    if (tag == "attribute") {
      if (!pend_has_) return kFallback;
      auto& table = (has_class_ && attr_class_ == "node") ? node_attr_ : edge_attr_;
      table[pend_id_] = pend_;
    } else if (tag == "attvalue") {
      if (kind_ == 0) return kOk;
      auto& table = kind_ == 1 ? node_attr_ : edge_attr_;
      if (!av_has_for_ || !av_has_value_) return kFallback;
      auto it = table.find(av_for_);
      if (it == table.end()) return kFallback;       // Python: "No attribute defined for="
      const AttrDef& d = it->second;
      if (!converts(d, av_value_)) return kFallback;
      if (kind_ == 1 && d.title == "node_type") {
        if (!stringy(d)) return kFallback;
        cur_type_ = av_value_;
        cur_has_type_ = true;
      } else if (kind_ == 2 && d.title == "label") {
        if (!stringy(d)) return kFallback;
        cur_att_rel_ = av_value_;
        cur_att_label_ = true;
      }
    } else if (tag == "node" && kind_ == 1) {
      const int32_t i = node_slot(cur_id_);
      g_.labels[i] = cur_label_;
      g_.label_null[i] = cur_label_null_ ? 1 : 0;
      if (cur_has_type_) g_.ntype[i] = intern(g_.type_map, &g_.type_names, cur_type_);
      kind_ = 0;
    } else if (tag == "edge" && kind_ == 2) {
      if (g_.directed && !cur_type_null_ && cur_etype_ == "undirected") return kFallback;
      if (!g_.directed && !cur_type_null_ && cur_etype_ == "directed") return kFallback;
      int32_t rel = -1;
      if (cur_att_label_) rel = intern(g_.rel_map, &g_.rel_names, cur_att_rel_);
      if (!cur_label_null_) rel = intern(g_.rel_map, &g_.rel_names, cur_label_);
      int64_t key = -1;
      if (!cur_key_null_) {
        key = static_cast<int64_t>(g_.key_buf.size());
        g_.key_buf.append(cur_key_);
        g_.key_buf.push_back('\0');
      }
      const int32_t s = node_slot(cur_src_), t = node_slot(cur_dst_);
      push(s, t, rel, key);
      if (!cur_type_null_ && cur_etype_ == "mutual") push(t, s, rel, key);
      kind_ = 0;
    } else if (tag == "nodes") {
      --depth_nodes_;
    }
    return kOk;
  }

  int32_t node_slot(const std::string& id) {
    auto it = g_.node_index.find(id);
    if (it != g_.node_index.end()) return it->second;
    const int32_t i = static_cast<int32_t>(g_.node_ids.size());
    g_.node_index.emplace(id, i);
    g_.node_ids.push_back(id);
    g_.labels.emplace_back();
    g_.label_null.push_back(1);
    g_.ntype.push_back(-1);
    return i;
  }
  void push(int32_t s, int32_t t, int32_t rel, int64_t key) {
    g_.e_src.push_back(s);
    g_.e_dst.push_back(t);
    g_.e_rel.push_back(rel);
    g_.key_off.push_back(key);
  }

  const char* p_;
  const char* e_;
  Gexf& g_;
  std::vector<Attr> attrs_;
  std::unordered_map<std::string, AttrDef> node_attr_, edge_attr_;
  std::string attr_class_;
  bool has_class_ = false;
  AttrDef pend_;
  std::string pend_id_;
  bool pend_has_ = false;
  int depth_nodes_ = 0;
  int kind_ = 0;   // 0 none, 1 node, 2 edge
  std::string cur_id_, cur_label_, cur_type_, cur_src_, cur_dst_, cur_key_, cur_etype_,
      cur_att_rel_;
  bool cur_label_null_ = true, cur_has_type_ = false, cur_key_null_ = true, cur_type_null_ = true,
       cur_att_label_ = false;
  std::string av_for_, av_value_;
  bool av_has_for_ = false, av_has_value_ = false, av_attrs_ok_ = false;
};

template <class V>
int64_t concat_bytes(const V& v) {
  int64_t n = 0;
  for (const auto& s : v) n += static_cast<int64_t>(s.size());
  return n;
}

template <class V>
void concat(const V& v, int64_t* off, char* buf) {
  int64_t o = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    off[i] = o;
    std::memcpy(buf + o, v[i].data(), v[i].size());
    o += static_cast<int64_t>(v[i].size());
  }
  off[v.size()] = o;
}

}  // namespace

extern "C" {

void* dps_gexf_open(const char* path, int32_t* status) {
  *status = kFallback;
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (::fstat(fd, &st) != 0) { ::close(fd); return nullptr; }
  const size_t n = static_cast<size_t>(st.st_size);
  void* m = n ? ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
  ::close(fd);
  if (n && m == MAP_FAILED) return nullptr;
  if (m) ::madvise(m, n, MADV_SEQUENTIAL);
  auto* g = new Gexf();
  g->node_index.reserve(n / 256 + 16);   // ~ one node per few hundred bytes of GEXF
  const char* b = static_cast<const char*>(m);
  Scanner sc(b, b + n, *g);
  *status = n ? sc.run() : kFallback;
  if (m) ::munmap(m, n);
  if (*status != kOk) { delete g; return nullptr; }
  return g;
}

// 0 nodes, 1 edges, 2 type names, 3 relationship names, 4 directed,
// 5 / 6 / 7 / 8 bytes of node ids / labels / type names / relationship names,
// 9 bytes of the edge-id buffer
int64_t dps_gexf_info(void* h, int32_t what) {
  const Gexf& g = *static_cast<const Gexf*>(h);
  switch (what) {
    case 0: return static_cast<int64_t>(g.node_ids.size());
    case 1: return static_cast<int64_t>(g.e_src.size());
    case 2: return static_cast<int64_t>(g.type_names.size());
    case 3: return static_cast<int64_t>(g.rel_names.size());
    case 4: return g.directed ? 1 : 0;
    case 5: return concat_bytes(g.node_ids);
    case 6: return concat_bytes(g.labels);
    case 7: return concat_bytes(g.type_names);
    case 8: return concat_bytes(g.rel_names);
    case 9: return static_cast<int64_t>(g.key_buf.size());
    default: return -1;
  }
}

int dps_gexf_export(void* h, int64_t* id_off, char* id_buf, int64_t* lab_off, char* lab_buf,
                    uint8_t* lab_null, int32_t* ntype, int64_t* type_off, char* type_buf,
                    int32_t* e_src, int32_t* e_dst, int32_t* e_rel, int64_t* e_key_off,
                    char* key_buf, int64_t* rel_off, char* rel_buf) {
  const Gexf& g = *static_cast<const Gexf*>(h);
  concat(g.node_ids, id_off, id_buf);
  concat(g.labels, lab_off, lab_buf);
  std::memcpy(lab_null, g.label_null.data(), g.label_null.size());
  std::memcpy(ntype, g.ntype.data(), g.ntype.size() * sizeof(int32_t));
  concat(g.type_names, type_off, type_buf);
  const size_t m = g.e_src.size() * sizeof(int32_t);
  std::memcpy(e_src, g.e_src.data(), m);
  std::memcpy(e_dst, g.e_dst.data(), m);
  std::memcpy(e_rel, g.e_rel.data(), m);
  std::memcpy(e_key_off, g.key_off.data(), g.key_off.size() * sizeof(int64_t));
  std::memcpy(key_buf, g.key_buf.data(), g.key_buf.size());
  concat(g.rel_names, rel_off, rel_buf);
  return 0;
}

void dps_gexf_close(void* h) { delete static_cast<Gexf*>(h); }

}  // extern "C"
