// model_io.hip — host-side reader of the unchanged XGBoost model file, so a C/C++/JNI caller can load
// the reference's model through the C-ABI alone (fd_load_xgboost_json).
//
// Reference: ml/models/model_manager.py:157-161 (_load_xgboost_model: XGBClassifier().load_model(path)),
// file written by ml/training/model_trainer.py:95-108 (XGBClassifier.save_model, XGBoost 2.0.3 JSON).
// Schema read: learner.objective.name (binary:logistic), learner.gradient_booster.{name (gbtree),
// model.trees[i].{left_children, right_children, split_indices, split_conditions, default_left, split_type,
// tree_param.size_leaf_vector}}, learner.learner_model_param.{base_score, num_feature, num_class}.
// A node is a leaf when left_children == -1; its weight is split_conditions (an f32 in XGBoost, printed
// round-trip exact). Same acceptance rules as the Python reader (fdengine/forest.py xgboost_from_json_doc).
// Numbers are converted with strtod (correctly rounded, as Python's float()).
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fd_internal.h"

namespace fd {
namespace {

// A small JSON DOM: arrays made only of numbers / booleans keep them in `nums` (model files are millions of
// such values), everything else is general.
struct JVal {
  enum Type { Null, Bool, Num, Str, Arr, Obj } type = Null;
  double num = 0.0;
  std::string str;
  std::vector<double> nums;  // Arr of numbers / booleans
  std::vector<JVal> arr;     // Arr of anything else
  std::vector<std::pair<std::string, JVal>> obj;
  bool numeric_array = false;

  const JVal* get(const char* key) const {
    if (type != Obj) return nullptr;
    for (const auto& kv : obj)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
};

struct Parser {
  const char* p;
  const char* end;
  [[noreturn]] void fail(const char* what) {
    throw Error(FD_ERR_INVALID_ARG, std::string("xgboost json: ") + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(const char* s) {
    const size_t n = std::strlen(s);
    if ((size_t)(end - p) >= n && std::memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  double number() {
    const char* a = p;
    if (p < end && (*p == '-' || *p == '+')) ++p;
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '-' || *p == '+'))
      ++p;
    if (p == a) fail("expected a number");
    char buf[64];
    const size_t n = (size_t)(p - a);
    if (n >= sizeof(buf)) fail("number too long");
    std::memcpy(buf, a, n);
    buf[n] = 0;
    char* e = nullptr;
    const double v = std::strtod(buf, &e);
    if (e != buf + n) fail("malformed number");
    return v;
  }
  std::string string() {
    if (p >= end || *p != '"') fail("expected a string");
    ++p;
    std::string s;
    while (p < end && *p != '"') {
      if (*p == '\\') {
        ++p;
        if (p >= end) fail("bad escape");
        const char c = *p++;
        switch (c) {
          case 'n': s += '\n'; break;
          case 't': s += '\t'; break;
          case 'r': s += '\r'; break;
          case 'b': s += '\b'; break;
          case 'f': s += '\f'; break;
          case 'u':  // names and values on the read path are ASCII; keep the code point's low byte
            if (end - p < 4) fail("bad \\u escape");
            s += (char)std::strtol(std::string(p, p + 4).c_str(), nullptr, 16);
            p += 4;
            break;
          default: s += c;
        }
      } else {
        s += *p++;
      }
    }
    if (p >= end) fail("unterminated string");
    ++p;
    return s;
  }
  JVal value(int depth) {
    if (depth > 64) fail("nesting too deep");
    ws();
    if (p >= end) fail("unexpected end of file");
    JVal v;
    const char c = *p;
    if (c == '{') {
      ++p;
      v.type = JVal::Obj;
      ws();
      if (p < end && *p == '}') {
        ++p;
        return v;
      }
      for (;;) {
        ws();
        std::string k = string();
        ws();
        if (p >= end || *p != ':') fail("expected ':'");
        ++p;
        v.obj.emplace_back(std::move(k), value(depth + 1));
        ws();
        if (p < end && *p == ',') {
          ++p;
          continue;
        }
        if (p < end && *p == '}') {
          ++p;
          return v;
        }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p;
      v.type = JVal::Arr;
      v.numeric_array = true;
      ws();
      if (p < end && *p == ']') {
        ++p;
        return v;
      }
      for (;;) {
        ws();
        if (p >= end) fail("unterminated array");
        const char d = *p;
        if (v.numeric_array && ((d >= '0' && d <= '9') || d == '-' || d == 't' || d == 'f')) {
          if (d == 't' || d == 'f') {
            const bool b = lit("true");
            if (!b && !lit("false")) fail("bad literal");
            v.nums.push_back(b ? 1.0 : 0.0);
          } else {
            v.nums.push_back(number());
          }
        } else {
          if (v.numeric_array) {  // mixed: demote the numbers read so far to general values
            for (double x : v.nums) {
              JVal n;
              n.type = JVal::Num;
              n.num = x;
              v.arr.push_back(std::move(n));
            }
            v.nums.clear();
            v.numeric_array = false;
          }
          v.arr.push_back(value(depth + 1));
        }
        ws();
        if (p < end && *p == ',') {
          ++p;
          continue;
        }
        if (p < end && *p == ']') {
          ++p;
          return v;
        }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.type = JVal::Str;
      v.str = string();
      return v;
    }
    if (lit("true")) {
      v.type = JVal::Bool;
      v.num = 1.0;
      return v;
    }
    if (lit("false")) {
      v.type = JVal::Bool;
      return v;
    }
    if (lit("null")) return v;
    v.type = JVal::Num;
    v.num = number();
    return v;
  }
};

const JVal& need(const JVal* v, const char* what) {
  if (!v) throw Error(FD_ERR_INVALID_ARG, std::string("xgboost json: missing ") + what);
  return *v;
}

// numbers may be stored as strings in learner_model_param ("5E-1", "64")
double as_num(const JVal& v, const char* what) {
  if (v.type == JVal::Num || v.type == JVal::Bool) return v.num;
  if (v.type == JVal::Str) {
    char* e = nullptr;
    const double x = std::strtod(v.str.c_str(), &e);
    if (e && *e == 0 && !v.str.empty()) return x;
  }
  throw Error(FD_ERR_INVALID_ARG, std::string("xgboost json: bad number in ") + what);
}

const std::vector<double>& num_array(const JVal& tree, const char* key) {
  const JVal& a = need(tree.get(key), key);
  if (a.type != JVal::Arr || (!a.numeric_array && !a.arr.empty()))
    throw Error(FD_ERR_INVALID_ARG, std::string("xgboost json: ") + key + " is not a numeric array");
  return a.nums;
}

}  // namespace

void read_xgboost_json(const char* path, XgbModel& out) {
  FD_REQUIRE(path != nullptr, FD_ERR_INVALID_ARG, "null path");
  std::FILE* f = std::fopen(path, "rb");
  FD_REQUIRE(f != nullptr, FD_ERR_IO, std::string("cannot open ") + path + ": " + std::strerror(errno));
  std::string text;
  {
    char buf[1 << 16];
    size_t r;
    while ((r = std::fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, r);
    const bool bad = std::ferror(f) != 0;
    std::fclose(f);
    FD_REQUIRE(!bad, FD_ERR_IO, std::string("read error on ") + path);
  }
  Parser ps{text.data(), text.data() + text.size()};
  const JVal doc = ps.value(0);
  const JVal& learner = need(doc.get("learner"), "learner");
  const JVal* obj = learner.get("objective");
  const JVal* oname = obj ? obj->get("name") : nullptr;
  FD_REQUIRE(oname && oname->type == JVal::Str && oname->str == "binary:logistic", FD_ERR_UNSUPPORTED,
             "objective " + (oname && oname->type == JVal::Str ? "'" + oname->str + "'" : std::string("None")) +
                 " not supported (binary:logistic only)");
  const JVal& gb = need(learner.get("gradient_booster"), "gradient_booster");
  const JVal* gname = gb.get("name");
  FD_REQUIRE(gname && gname->type == JVal::Str && gname->str == "gbtree", FD_ERR_UNSUPPORTED,
             "booster not supported (gbtree only)");
  const JVal& lmp = need(learner.get("learner_model_param"), "learner_model_param");
  const JVal* nc = lmp.get("num_class");
  FD_REQUIRE(!nc || (int)as_num(*nc, "num_class") <= 1, FD_ERR_UNSUPPORTED, "multi-class models are not supported");
  out.num_feature = (int)as_num(need(lmp.get("num_feature"), "num_feature"), "num_feature");
  out.base_score = as_num(need(lmp.get("base_score"), "base_score"), "base_score");
  const JVal& trees = need(need(gb.get("model"), "model").get("trees"), "trees");
  FD_REQUIRE(trees.type == JVal::Arr && !trees.numeric_array, FD_ERR_INVALID_ARG, "xgboost json: trees is not a list");
  out.offsets.assign(1, 0);
  out.left.clear();
  out.right.clear();
  out.feature.clear();
  out.threshold.clear();
  out.default_left.clear();
  out.leaf_value.clear();
  for (const JVal& tr : trees.arr) {
    const auto& L = num_array(tr, "left_children");
    const auto& R = num_array(tr, "right_children");
    const auto& F = num_array(tr, "split_indices");
    const auto& C = num_array(tr, "split_conditions");
    const auto& DL = num_array(tr, "default_left");
    const size_t m = L.size();
    FD_REQUIRE(R.size() == m && F.size() == m && C.size() == m && DL.size() == m, FD_ERR_INVALID_ARG,
               "xgboost json: tree arrays of different lengths");
    if (const JVal* st = tr.get("split_type")) {
      FD_REQUIRE(st->type == JVal::Arr && st->numeric_array, FD_ERR_INVALID_ARG, "xgboost json: bad split_type");
      for (double x : st->nums) FD_REQUIRE(x == 0.0, FD_ERR_UNSUPPORTED, "categorical splits are not supported");
    }
    if (const JVal* tp = tr.get("tree_param"))
      if (const JVal* slv = tp->get("size_leaf_vector"))
        FD_REQUIRE((int)as_num(*slv, "size_leaf_vector") <= 1, FD_ERR_UNSUPPORTED, "vector leaves are not supported");
    for (size_t i = 0; i < m; ++i) {
      const bool leaf = L[i] == -1.0;
      out.left.push_back(leaf ? -1 : (int32_t)L[i]);
      out.right.push_back((int32_t)R[i]);
      out.feature.push_back(leaf ? 0 : (int32_t)F[i]);
      out.threshold.push_back(leaf ? 0.0 : C[i]);
      out.default_left.push_back(DL[i] != 0.0 ? 1 : 0);
      out.leaf_value.push_back(leaf ? (double)(float)C[i] : 0.0);  // XGBoost holds node values as f32
    }
    out.offsets.push_back((int64_t)out.left.size());
  }
}

}  // namespace fd
