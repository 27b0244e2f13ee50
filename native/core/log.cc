#include "core/log.h"

#include <sys/time.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string_view>
#include <utility>
#include <vector>

namespace p2pt::log {
namespace {

struct Directive {
  std::string prefix;  // empty == global default
  Level level;
};

std::vector<Directive> g_directives;
Level g_default = Level::Info;
Level g_max = Level::Info;  // fast-path: most verbose level of any directive

bool parse_level(std::string_view s, Level& out) {
  std::string l(s);
  for (auto& c : l) c = char(tolower(c));
  if (l == "error") out = Level::Error;
  else if (l == "warn" || l == "warning") out = Level::Warn;
  else if (l == "info") out = Level::Info;
  else if (l == "debug") out = Level::Debug;
  else if (l == "trace") out = Level::Trace;
  else if (l == "off") out = Level(0);
  else return false;
  return true;
}

const char* level_name(Level l) {
  switch (l) {
    case Level::Error: return "ERROR";
    case Level::Warn: return " WARN";
    case Level::Info: return " INFO";
    case Level::Debug: return "DEBUG";
    case Level::Trace: return "TRACE";
  }
  return "?";
}

}  // namespace

void init(const std::string& spec_in) {
  g_directives.clear();
  g_default = Level::Info;
  std::string spec = spec_in.empty() ? "info" : spec_in;
  size_t start = 0;
  while (start <= spec.size()) {
    size_t comma = spec.find(',', start);
    if (comma == std::string::npos) comma = spec.size();
    std::string_view d(spec.data() + start, comma - start);
    start = comma + 1;
    if (d.empty()) continue;
    size_t eq = d.find('=');
    Level lvl;
    if (eq == std::string_view::npos) {
      if (parse_level(d, lvl)) g_default = lvl;
      else g_directives.push_back({std::string(d), Level::Trace});  // bare target => all
    } else if (parse_level(d.substr(eq + 1), lvl)) {
      g_directives.push_back({std::string(d.substr(0, eq)), lvl});
    }
  }
  g_max = g_default;
  for (auto& d : g_directives)
    if (int(d.level) > int(g_max)) g_max = d.level;
}

void init_from_env() {
  const char* s = getenv("TUNNEL_LOG");
  if (!s || !*s) s = getenv("RUST_LOG");
  init(s ? s : "");
}

bool enabled(Level lvl, const char* target) {
  if (int(lvl) > int(g_max)) return false;
  Level eff = g_default;
  size_t best = 0;
  for (auto& d : g_directives) {
    // Accept the reference crate name "tunnel" and "p2pt" interchangeably.
    if (strncmp(target, d.prefix.c_str(), d.prefix.size()) == 0 && d.prefix.size() >= best) {
      best = d.prefix.size();
      eff = d.level;
    }
  }
  return int(lvl) <= int(eff);
}

void vwrite(Level lvl, const char* target, const char* fmt, va_list ap) {
  char msg[4096];
  vsnprintf(msg, sizeof msg, fmt, ap);
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  struct tm tm;
  gmtime_r(&tv.tv_sec, &tm);
  char ts[64];
  strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%S", &tm);
  // One fwrite per line so concurrent writers (forks) never interleave mid-line.
  char line[4352];
  int n = snprintf(line, sizeof line, "%s.%06ldZ %s %s: %s\n", ts, long(tv.tv_usec),
                   level_name(lvl), target, msg);
  if (n > int(sizeof line)) n = sizeof line;
  fwrite(line, 1, size_t(n), stdout);
  fflush(stdout);
}

void write(Level lvl, const char* target, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vwrite(lvl, target, fmt, ap);
  va_end(ap);
}

}  // namespace p2pt::log
