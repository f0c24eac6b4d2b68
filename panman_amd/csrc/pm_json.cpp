// pm_json.cpp -- recursive-descent JSON reader (RFC 8259 subset: no comments; \u escapes
// outside the BMP are kept as UTF-8 of each surrogate, which PanGraph files never hold).
#include "pm_json.h"

#include <cstdlib>
#include <cstring>

namespace pm {

namespace {

const Json kNullJson{};
const std::string kEmpty;

struct Parser {
    const std::string& s;
    size_t i = 0;
    std::string err;
    int depth = 0;

    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool fail(const char* what) {
        if (err.empty()) err = std::string(what) + " at byte " + std::to_string(i);
        return false;
    }
    bool lit(const char* w) {
        const size_t n = std::strlen(w);
        if (s.compare(i, n, w) != 0) return fail("bad literal");
        i += n;
        return true;
    }
    static void utf8(uint32_t cp, std::string& o) {
        if (cp < 0x80) {
            o += (char)cp;
        } else if (cp < 0x800) {
            o += (char)(0xC0 | (cp >> 6));
            o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xE0 | (cp >> 12));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        }
    }
    bool string(std::string& o) {
        if (i >= s.size() || s[i] != '"') return fail("expected string");
        ++i;
        while (true) {
            if (i >= s.size()) return fail("unterminated string");
            const char c = s[i++];
            if (c == '"') return true;
            if (c != '\\') {
                o += c;
                continue;
            }
            if (i >= s.size()) return fail("bad escape");
            const char e = s[i++];
            switch (e) {
                case '"': o += '"'; break;
                case '\\': o += '\\'; break;
                case '/': o += '/'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'n': o += '\n'; break;
                case 'r': o += '\r'; break;
                case 't': o += '\t'; break;
                case 'u': {
                    if (i + 4 > s.size()) return fail("bad \\u escape");
                    uint32_t cp = 0;
                    for (int k = 0; k < 4; ++k) {
                        const char h = s[i++];
                        cp <<= 4;
                        if (h >= '0' && h <= '9') cp |= h - '0';
                        else if (h >= 'a' && h <= 'f') cp |= h - 'a' + 10;
                        else if (h >= 'A' && h <= 'F') cp |= h - 'A' + 10;
                        else return fail("bad \\u escape");
                    }
                    utf8(cp, o);
                    break;
                }
                default: return fail("bad escape");
            }
        }
    }
    bool number(Json& v) {
        const size_t b = i;
        if (i < s.size() && s[i] == '-') ++i;
        bool frac = false;
        while (i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                                s[i] == '+' || s[i] == '-')) {
            frac |= s[i] == '.' || s[i] == 'e' || s[i] == 'E';
            ++i;
        }
        if (i == b) return fail("expected value");
        const std::string t = s.substr(b, i - b);
        v.kind = Json::kNumber;
        char* end = nullptr;
        v.num = std::strtod(t.c_str(), &end);
        if (end != t.c_str() + t.size()) return fail("bad number");
        if (!frac) {
            v.inum = std::strtoll(t.c_str(), nullptr, 10);
            v.is_int = true;
        }
        return true;
    }
    bool value(Json& v) {
        if (++depth > 512) return fail("nesting too deep");
        ws();
        if (i >= s.size()) return fail("unexpected end");
        bool ok = true;
        const char c = s[i];
        if (c == '{') {
            v.kind = Json::kObject;
            ++i;
            ws();
            if (i < s.size() && s[i] == '}') {
                ++i;
            } else {
                while (ok) {
                    ws();
                    std::string k;
                    if (!string(k)) return false;
                    ws();
                    if (i >= s.size() || s[i] != ':') return fail("expected ':'");
                    ++i;
                    Json& slot = v.obj[k];
                    slot = Json{};
                    if (!value(slot)) return false;
                    ws();
                    if (i < s.size() && s[i] == ',') { ++i; continue; }
                    if (i < s.size() && s[i] == '}') { ++i; break; }
                    return fail("expected ',' or '}'");
                }
            }
        } else if (c == '[') {
            v.kind = Json::kArray;
            ++i;
            ws();
            if (i < s.size() && s[i] == ']') {
                ++i;
            } else {
                while (true) {
                    v.arr.emplace_back();
                    if (!value(v.arr.back())) return false;
                    ws();
                    if (i < s.size() && s[i] == ',') { ++i; continue; }
                    if (i < s.size() && s[i] == ']') { ++i; break; }
                    return fail("expected ',' or ']'");
                }
            }
        } else if (c == '"') {
            v.kind = Json::kString;
            ok = string(v.str);
        } else if (c == 't') {
            v.kind = Json::kBool;
            v.b = true;
            ok = lit("true");
        } else if (c == 'f') {
            v.kind = Json::kBool;
            ok = lit("false");
        } else if (c == 'n') {
            v.kind = Json::kNull;
            ok = lit("null");
        } else {
            ok = number(v);
        }
        --depth;
        return ok;
    }
};

}  // namespace

const Json& Json::operator[](const std::string& k) const {
    if (kind != kObject) return kNullJson;
    auto it = obj.find(k);
    return it == obj.end() ? kNullJson : it->second;
}

const Json& Json::operator[](size_t i) const { return kind == kArray && i < arr.size() ? arr[i] : kNullJson; }

const std::string& Json::as_string() const { return kind == kString ? str : kEmpty; }

bool json_parse(const std::string& text, Json& out, std::string& err) {
    Parser p{text};
    out = Json{};
    if (!p.value(out)) {
        err = p.err;
        return false;
    }
    p.ws();
    if (p.i != text.size()) {
        err = "trailing characters at byte " + std::to_string(p.i);
        return false;
    }
    return true;
}

}  // namespace pm
