// vpt_config.cpp — strict reader for the reference's scene JSON (include/vpt/configuration.hpp:14-65).
//
// The reference reads the file with glaze, `glz::read_file_json<{.error_on_missing_keys = true}>`
// (src/configuration.cpp:8-22); glaze's default also rejects unknown keys.  On error the reference
// calls vptFATAL (exit(1)); here the error is returned (VPT_E_PARSE / VPT_E_IO) with a message.
// Floats are parsed straight to the nearest float (strtof), integers must be non-negative where the
// reference field is unsigned.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "vpt_internal.h"

namespace vpt {
namespace {

struct JVal {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  std::string text;  // number text or string value
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
};

struct Parser {
  const char* p;
  const char* end;
  std::string err;
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool fail(const std::string& m) {
    if (err.empty()) err = m;
    return false;
  }
  bool parse_string(std::string& s) {
    if (p >= end || *p != '"') return fail("expected string");
    ++p;
    while (p < end && *p != '"') {
      char c = *p++;
      if (c == '\\') {
        if (p >= end) return fail("bad escape");
        char e = *p++;
        switch (e) {
          case '"': s += '"'; break;
          case '\\': s += '\\'; break;
          case '/': s += '/'; break;
          case 'b': s += '\b'; break;
          case 'f': s += '\f'; break;
          case 'n': s += '\n'; break;
          case 'r': s += '\r'; break;
          case 't': s += '\t'; break;
          case 'u': {
            if (end - p < 4) return fail("bad \\u escape");
            unsigned v = (unsigned)std::strtoul(std::string(p, 4).c_str(), nullptr, 16);
            p += 4;
            if (v < 0x80) {
              s += (char)v;
            } else if (v < 0x800) {
              s += (char)(0xC0 | (v >> 6));
              s += (char)(0x80 | (v & 0x3F));
            } else {
              s += (char)(0xE0 | (v >> 12));
              s += (char)(0x80 | ((v >> 6) & 0x3F));
              s += (char)(0x80 | (v & 0x3F));
            }
            break;
          }
          default: return fail("bad escape");
        }
      } else {
        s += c;
      }
    }
    if (p >= end) return fail("unterminated string");
    ++p;
    return true;
  }
  bool parse(JVal& v, int depth = 0) {
    if (depth > 64) return fail("nesting too deep");
    ws();
    if (p >= end) return fail("unexpected end of input");
    char c = *p;
    if (c == '{') {
      ++p;
      v.kind = JVal::Obj;
      ws();
      if (p < end && *p == '}') {
        ++p;
        return true;
      }
      while (true) {
        ws();
        std::string key;
        if (!parse_string(key)) return false;
        ws();
        if (p >= end || *p != ':') return fail("expected ':'");
        ++p;
        JVal child;
        if (!parse(child, depth + 1)) return false;
        v.obj.emplace_back(std::move(key), std::move(child));
        ws();
        if (p < end && *p == ',') {
          ++p;
          continue;
        }
        if (p < end && *p == '}') {
          ++p;
          return true;
        }
        return fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p;
      v.kind = JVal::Arr;
      ws();
      if (p < end && *p == ']') {
        ++p;
        return true;
      }
      while (true) {
        JVal child;
        if (!parse(child, depth + 1)) return false;
        v.arr.push_back(std::move(child));
        ws();
        if (p < end && *p == ',') {
          ++p;
          continue;
        }
        if (p < end && *p == ']') {
          ++p;
          return true;
        }
        return fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.kind = JVal::Str;
      return parse_string(v.text);
    }
    if (end - p >= 4 && std::strncmp(p, "true", 4) == 0) {
      p += 4;
      v.kind = JVal::Bool;
      v.b = true;
      return true;
    }
    if (end - p >= 5 && std::strncmp(p, "false", 5) == 0) {
      p += 5;
      v.kind = JVal::Bool;
      v.b = false;
      return true;
    }
    if (end - p >= 4 && std::strncmp(p, "null", 4) == 0) {
      p += 4;
      v.kind = JVal::Null;
      return true;
    }
    const char* s = p;
    if (p < end && (*p == '-' || *p == '+')) ++p;
    while (p < end && (std::isdigit((unsigned char)*p) || *p == '.' || *p == 'e' || *p == 'E' || *p == '-' || *p == '+')) ++p;
    if (p == s) return fail(std::string("unexpected character '") + c + "'");
    v.kind = JVal::Num;
    v.text.assign(s, p);
    return true;
  }
};

struct Reader {
  std::string err;
  bool fail(const std::string& m) {
    if (err.empty()) err = m;
    return false;
  }
  // Object with exactly the keys in `keys` (error_on_missing_keys + unknown keys rejected).
  bool object(const JVal& v, const std::string& where, std::initializer_list<const char*> keys,
              std::map<std::string, const JVal*>& out) {
    if (v.kind != JVal::Obj) return fail(where + ": expected an object");
    for (auto& kv : v.obj) {
      bool known = false;
      for (const char* k : keys) known |= (kv.first == k);
      if (!known) return fail(where + ": unknown key \"" + kv.first + "\"");
      out[kv.first] = &kv.second;
    }
    for (const char* k : keys)
      if (!out.count(k)) return fail(where + ": missing key \"" + std::string(k) + "\"");
    return true;
  }
  bool f32(const JVal* v, const std::string& where, float& out) {
    if (v->kind != JVal::Num) return fail(where + ": expected a number");
    char* e = nullptr;
    errno = 0;
    float x = std::strtof(v->text.c_str(), &e);
    if (!e || *e) return fail(where + ": bad number '" + v->text + "'");
    out = x;
    return true;
  }
  bool i64(const JVal* v, const std::string& where, int64_t& out, bool non_negative) {
    if (v->kind != JVal::Num) return fail(where + ": expected an integer");
    char* e = nullptr;
    errno = 0;
    long long x = std::strtoll(v->text.c_str(), &e, 10);
    if (!e || *e || errno) return fail(where + ": expected an integer, got '" + v->text + "'");
    if (non_negative && x < 0) return fail(where + ": expected a non-negative integer");
    out = x;
    return true;
  }
  bool u32(const JVal* v, const std::string& where, uint32_t& out) {
    int64_t x;
    if (!i64(v, where, x, true)) return false;
    if (x > 0xFFFFFFFFLL) return fail(where + ": out of range for unsigned int");
    out = (uint32_t)x;
    return true;
  }
  bool boolean(const JVal* v, const std::string& where, int32_t& out) {
    if (v->kind != JVal::Bool) return fail(where + ": expected true/false");
    out = v->b ? 1 : 0;
    return true;
  }
  bool vec3(const JVal* v, const std::string& where, float out[3]) {
    if (v->kind != JVal::Arr || v->arr.size() != 3) return fail(where + ": expected an array of 3 numbers");
    for (int i = 0; i < 3; ++i)
      if (!f32(&v->arr[i], where, out[i])) return false;
    return true;
  }
  bool size2(const JVal* v, const std::string& where, int64_t out[2]) {
    if (v->kind != JVal::Arr || v->arr.size() != 2) return fail(where + ": expected an array of 2 integers");
    for (int i = 0; i < 2; ++i)
      if (!i64(&v->arr[i], where, out[i], false)) return false;
    return true;
  }
};

int parse_config(const char* text, size_t len, vpt_configuration* out) {
  Parser P{text, text + len, {}};
  JVal root;
  if (!P.parse(root)) return set_error(VPT_E_PARSE, "configuration JSON: " + P.err);
  P.ws();
  if (P.p != P.end) return set_error(VPT_E_PARSE, "configuration JSON: trailing characters");
  Reader R;
  vpt_configuration c;
  std::memset(&c, 0, sizeof c);
  std::map<std::string, const JVal*> top, cam, wk, sp, il, dl, vol;
  bool ok = R.object(root, "configuration",
                     {"seed", "output_size", "tile_size", "num_waves", "num_workers", "camera_parameters",
                      "worker_parameters", "volume_path", "volume_parameters"},
                     top) &&
            R.u32(top["seed"], "seed", c.seed) && R.size2(top["output_size"], "output_size", c.output_size) &&
            R.size2(top["tile_size"], "tile_size", c.tile_size) && R.u32(top["num_waves"], "num_waves", c.num_waves) &&
            R.u32(top["num_workers"], "num_workers", c.num_workers);
  ok = ok && R.object(*top["camera_parameters"], "camera_parameters",
                      {"position", "look", "up", "vfov_deg", "imaging_ratio"}, cam) &&
       R.vec3(cam["position"], "camera_parameters.position", c.camera_parameters.position) &&
       R.vec3(cam["look"], "camera_parameters.look", c.camera_parameters.look) &&
       R.vec3(cam["up"], "camera_parameters.up", c.camera_parameters.up) &&
       R.f32(cam["vfov_deg"], "camera_parameters.vfov_deg", c.camera_parameters.vfov_deg) &&
       R.f32(cam["imaging_ratio"], "camera_parameters.imaging_ratio", c.camera_parameters.imaging_ratio);
  vpt_worker_params& w = c.worker_parameters;
  ok = ok && R.object(*top["worker_parameters"], "worker_parameters",
                      {"single_pixel", "use_jitter", "infinite_light", "distant_light", "max_depth"}, wk) &&
       R.object(*wk["single_pixel"], "worker_parameters.single_pixel", {"enabled", "coord"}, sp) &&
       R.boolean(sp["enabled"], "single_pixel.enabled", w.single_pixel_enabled) &&
       R.size2(sp["coord"], "single_pixel.coord", w.single_pixel_coord) &&
       R.boolean(wk["use_jitter"], "worker_parameters.use_jitter", w.use_jitter) &&
       R.object(*wk["infinite_light"], "worker_parameters.infinite_light", {"xyz", "multiplier"}, il) &&
       R.vec3(il["xyz"], "infinite_light.xyz", w.infinite_light_xyz) &&
       R.f32(il["multiplier"], "infinite_light.multiplier", w.infinite_light_multiplier) &&
       R.object(*wk["distant_light"], "worker_parameters.distant_light", {"xyz", "multiplier", "inv_direction"}, dl) &&
       R.vec3(dl["xyz"], "distant_light.xyz", w.distant_light_xyz) &&
       R.f32(dl["multiplier"], "distant_light.multiplier", w.distant_light_multiplier) &&
       R.vec3(dl["inv_direction"], "distant_light.inv_direction", w.distant_light_inv_direction) &&
       R.u32(wk["max_depth"], "worker_parameters.max_depth", w.max_depth);
  vpt_volume_params& v = c.volume_parameters;
  ok = ok && R.object(*top["volume_parameters"], "volume_parameters",
                      {"henyey_greenstein_g", "le_scale", "sigma_a", "sigma_s", "temperature_offset", "temperature_scale"},
                      vol) &&
       R.f32(vol["henyey_greenstein_g"], "volume_parameters.henyey_greenstein_g", v.henyey_greenstein_g) &&
       R.f32(vol["le_scale"], "volume_parameters.le_scale", v.le_scale) &&
       R.f32(vol["sigma_a"], "volume_parameters.sigma_a", v.sigma_a) &&
       R.f32(vol["sigma_s"], "volume_parameters.sigma_s", v.sigma_s) &&
       R.f32(vol["temperature_offset"], "volume_parameters.temperature_offset", v.temperature_offset) &&
       R.f32(vol["temperature_scale"], "volume_parameters.temperature_scale", v.temperature_scale);
  if (ok) {
    const JVal* vp = top["volume_path"];
    if (vp->kind != JVal::Str) {
      ok = R.fail("volume_path: expected a string");
    } else if (vp->text.size() >= sizeof c.volume_path) {
      ok = R.fail("volume_path: too long");
    } else {
      std::memcpy(c.volume_path, vp->text.c_str(), vp->text.size() + 1);
    }
  }
  if (!ok) return set_error(VPT_E_PARSE, "configuration: " + R.err);
  *out = c;
  return VPT_OK;
}

}  // namespace
}  // namespace vpt

extern "C" int vpt_config_parse(const char* json_text, size_t len, vpt_configuration* out) {
  if (!json_text || !out) return vpt::set_error(VPT_E_INVALID, "vpt_config_parse: null argument");
  return vpt::parse_config(json_text, len, out);
}

extern "C" int vpt_config_read(const char* path, vpt_configuration* out) {
  if (!path || !out) return vpt::set_error(VPT_E_INVALID, "vpt_config_read: null argument");
  std::ifstream f(path, std::ios::binary);
  if (!f) return vpt::set_error(VPT_E_IO, std::string("cannot read configuration file \"") + path + "\"");
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  return vpt::parse_config(s.data(), s.size(), out);
}
