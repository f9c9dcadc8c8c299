#include <qmf/utils/Flags.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <vector>

namespace qmf {
namespace flags {

std::map<std::string, Flag>& registry() {
  static std::map<std::string, Flag> r;
  return r;
}

Registrar::Registrar(const char* name, Kind kind, void* ptr, const char* help,
                     const std::string& def) {
  registry()[name] = Flag{kind, ptr, help, def};
}

static bool parseBool(const std::string& v, bool* out) {
  if (v == "true" || v == "1" || v == "yes" || v == "t" || v == "y") {
    *out = true;
    return true;
  }
  if (v == "false" || v == "0" || v == "no" || v == "f" || v == "n") {
    *out = false;
    return true;
  }
  return false;
}

std::string set(const std::string& name, const std::string& value) {
  auto it = registry().find(name);
  if (it == registry().end()) return "unknown command line flag '" + name + "'";
  Flag& f = it->second;
  const char* s = value.c_str();
  char* end = nullptr;
  errno = 0;
  switch (f.kind) {
    case Kind::Bool: {
      bool b;
      if (!parseBool(value, &b)) return "illegal value '" + value + "' for bool flag " + name;
      *static_cast<bool*>(f.ptr) = b;
      return "";
    }
    case Kind::Int32: {
      long v = std::strtol(s, &end, 10);
      if (end == s || *end || errno || v < INT32_MIN || v > INT32_MAX)
        return "illegal value '" + value + "' for int32 flag " + name;
      *static_cast<int32_t*>(f.ptr) = (int32_t)v;
      return "";
    }
    case Kind::UInt64: {
      if (!value.empty() && value[0] == '-') return "illegal value '" + value + "' for uint64 flag " + name;
      unsigned long long v = std::strtoull(s, &end, 10);
      if (end == s || *end || errno) return "illegal value '" + value + "' for uint64 flag " + name;
      *static_cast<uint64_t*>(f.ptr) = (uint64_t)v;
      return "";
    }
    case Kind::Double: {
      double v = std::strtod(s, &end);
      if (end == s || *end) return "illegal value '" + value + "' for double flag " + name;
      *static_cast<double*>(f.ptr) = v;
      return "";
    }
    case Kind::String:
      *static_cast<std::string*>(f.ptr) = value;
      return "";
  }
  return "bad flag kind";
}

std::string usage(const std::string& program) {
  std::ostringstream os;
  os << program << "\n  Flags:\n";
  for (const auto& kv : registry()) {
    os << "    -" << kv.first << " (" << kv.second.help << ") default: " << kv.second.defval
       << "\n";
  }
  return os.str();
}

bool parse(int* argc, char*** argv, const std::string& program) {
  std::vector<char*> rest;
  rest.push_back((*argv)[0]);
  for (int i = 1; i < *argc; ++i) {
    std::string a = (*argv)[i];
    if (a.size() < 2 || a[0] != '-') {
      rest.push_back((*argv)[i]);
      continue;
    }
    if (a == "--") {
      for (int j = i + 1; j < *argc; ++j) rest.push_back((*argv)[j]);
      break;
    }
    std::string body = a.substr(a[1] == '-' ? 2 : 1);
    if (body == "help" || body == "helpfull") {
      std::cerr << usage(program);
      return false;
    }
    std::string name = body, value;
    bool has_value = false;
    const auto eq = body.find('=');
    if (eq != std::string::npos) {
      name = body.substr(0, eq);
      value = body.substr(eq + 1);
      has_value = true;
    }
    auto it = registry().find(name);
    if (it == registry().end() && !has_value && name.rfind("no", 0) == 0) {
      auto it2 = registry().find(name.substr(2));
      if (it2 != registry().end() && it2->second.kind == Kind::Bool) {
        *static_cast<bool*>(it2->second.ptr) = false;
        continue;
      }
    }
    if (it == registry().end()) {
      std::cerr << "ERROR: unknown command line flag '" << name << "'\n";
      std::exit(1);
    }
    if (!has_value) {
      if (it->second.kind == Kind::Bool) {
        value = "true";
      } else if (i + 1 < *argc) {
        value = (*argv)[++i];
      } else {
        std::cerr << "ERROR: flag '" << a << "' is missing its argument\n";
        std::exit(1);
      }
    }
    const std::string err = set(name, value);
    if (!err.empty()) {
      std::cerr << "ERROR: " << err << "\n";
      std::exit(1);
    }
  }
  static std::vector<char*> keep;
  keep = rest;
  keep.push_back(nullptr);
  *argc = (int)rest.size();
  *argv = keep.data();
  return true;
}

}  // namespace flags
}  // namespace qmf
