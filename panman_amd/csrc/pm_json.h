// pm_json.h -- minimal JSON reader for PanGraph files (the reference reads them with
// jsoncpp, src/panman.cpp:825-826).  Objects keep their members sorted by key, as
// Json::Value::getMemberNames returns them; missing members and null read as 0 / "" /
// false / empty, as jsoncpp's const accessors do.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace pm {

struct Json {
    enum Kind { kNull, kBool, kNumber, kString, kArray, kObject } kind = kNull;
    bool b = false;
    double num = 0;
    int64_t inum = 0;
    bool is_int = false;
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    const Json& operator[](const std::string& k) const;
    const Json& operator[](size_t i) const;
    size_t size() const { return kind == kArray ? arr.size() : kind == kObject ? obj.size() : 0; }
    int64_t as_int() const { return kind == kNumber ? (is_int ? inum : (int64_t)num) : (kind == kBool ? b : 0); }
    bool as_bool() const { return kind == kBool ? b : (kind == kNumber ? as_int() != 0 : false); }
    const std::string& as_string() const;
};

// Parse `text`; on failure returns false and sets `err` (with the byte offset).
bool json_parse(const std::string& text, Json& out, std::string& err);

}  // namespace pm
