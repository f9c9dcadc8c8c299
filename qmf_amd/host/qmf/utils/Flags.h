// Command-line flags with gflags' syntax, so the reference's command lines work unchanged
// (wals.cpp:26-50, bpr.cpp:28-59): -name=value, --name=value, --name value, and for
// booleans --name, --noname, --name=true|false|1|0.  Unknown flags abort with a message.
#pragma once

#include <cstdint>
#include <map>
#include <string>

namespace qmf {
namespace flags {

enum class Kind { Bool, Int32, UInt64, Double, String };

struct Flag {
  Kind kind;
  void* ptr;
  std::string help;
  std::string defval;
};

std::map<std::string, Flag>& registry();

struct Registrar {
  Registrar(const char* name, Kind kind, void* ptr, const char* help, const std::string& def);
};

// Parses and removes recognised flags from argv.  Returns false on --help (usage printed).
bool parse(int* argc, char*** argv, const std::string& usage);
// Sets one flag from text; returns an error message or "" on success.
std::string set(const std::string& name, const std::string& value);
std::string usage(const std::string& program);

}  // namespace flags
}  // namespace qmf

#define QMF_FLAG_DEF(type, kind, name, def, help)                                          \
  type FLAGS_##name = def;                                                                 \
  static ::qmf::flags::Registrar qmf_flag_reg_##name(#name, ::qmf::flags::Kind::kind,      \
                                                     &FLAGS_##name, help, #def)

#define DEFINE_bool(name, def, help) QMF_FLAG_DEF(bool, Bool, name, def, help)
#define DEFINE_int32(name, def, help) QMF_FLAG_DEF(int32_t, Int32, name, def, help)
#define DEFINE_uint64(name, def, help) QMF_FLAG_DEF(uint64_t, UInt64, name, def, help)
#define DEFINE_double(name, def, help) QMF_FLAG_DEF(double, Double, name, def, help)
#define DEFINE_string(name, def, help) QMF_FLAG_DEF(std::string, String, name, def, help)
