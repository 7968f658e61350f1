// json_min.h — a small DOM JSON parser for the scene files (scenes/*.json).
// Numbers keep their source text so f32 fields are parsed with strtof (correctly
// rounded, as serde_json's f32 parse in basics/scene_loader.rs:3-7), not via double.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace fr {
namespace json {

struct Value {
  enum Type { Null, Bool, Number, String, Array, Object } type = Null;
  bool b = false;
  std::string text;  // number source text or string contents
  std::vector<Value> items;
  std::vector<std::pair<std::string, Value>> members;  // insertion order kept

  const Value* get(const char* key) const {
    for (const auto& kv : members)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
};

// Returns true on success; on failure `err` holds a message with the byte offset.
bool parse(const char* text, size_t len, Value& out, std::string& err);

}  // namespace json
}  // namespace fr
