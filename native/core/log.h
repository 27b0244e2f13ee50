// Leveled logging with an env-var filter.
//
// Mirrors the reference's tracing_subscriber setup (reference
// tunnel/src/main.rs:21-25): the filter is read from RUST_LOG (or TUNNEL_LOG),
// default "info"; directives look like "debug" or "info,tunnel::serve=debug".
// Lines go to stdout in the tracing fmt layout
//   2026-02-06T10:00:00.123456Z  INFO tunnel::serve: sent AGREE, tunnel ready
// because the e2e scripts grep these strings (reference scripts/test-tunnel.sh:79-86).
#pragma once

#include <cstdarg>
#include <string>

namespace p2pt::log {

enum class Level : int { Error = 1, Warn = 2, Info = 3, Debug = 4, Trace = 5 };

// Parse a filter spec (e.g. "info,tunnel::rtc=trace"). Empty -> "info".
void init(const std::string& spec);
// init() from RUST_LOG / TUNNEL_LOG.
void init_from_env();
bool enabled(Level lvl, const char* target);
void write(Level lvl, const char* target, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
void vwrite(Level lvl, const char* target, const char* fmt, va_list ap);

}  // namespace p2pt::log

#define P2PT_LOG(lvl, target, ...)                                         \
  do {                                                                     \
    if (::p2pt::log::enabled(lvl, target)) ::p2pt::log::write(lvl, target, __VA_ARGS__); \
  } while (0)
#define LOG_ERROR(target, ...) P2PT_LOG(::p2pt::log::Level::Error, target, __VA_ARGS__)
#define LOG_WARN(target, ...) P2PT_LOG(::p2pt::log::Level::Warn, target, __VA_ARGS__)
#define LOG_INFO(target, ...) P2PT_LOG(::p2pt::log::Level::Info, target, __VA_ARGS__)
#define LOG_DEBUG(target, ...) P2PT_LOG(::p2pt::log::Level::Debug, target, __VA_ARGS__)
#define LOG_TRACE(target, ...) P2PT_LOG(::p2pt::log::Level::Trace, target, __VA_ARGS__)
