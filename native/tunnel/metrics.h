// Counters, gauges, a Prometheus text endpoint, and per-stream trace events.
//
// The reference has logging only. These are additive and
// off the wire: the /metrics endpoint is only served with --metrics-listen,
// and trace events are only written when TUNNEL_TRACE=<path> is set (JSONL
// with monotonic microsecond timestamps, used to measure added TTFT).
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>

#include "core/net.h"
#include "core/reactor.h"

namespace p2pt::metrics {

void frame_sent(uint8_t type, size_t bytes);
void frame_recv(uint8_t type, size_t bytes);
void counter_add(const std::string& name, double v = 1);
void gauge_set(const std::string& name, double v);
// Lazily evaluated gauge (e.g. SCTP cwnd); replaced if the name exists.
void gauge_fn(const std::string& name, std::function<double()> fn);
void gauge_fn_remove(const std::string& name);
double counter_get(const std::string& name);
std::string render_prometheus();

// Serves GET /metrics on addr until the returned handle is destroyed.
std::shared_ptr<void> serve(Reactor& r, const std::string& addr, std::string* err);

}  // namespace p2pt::metrics

namespace p2pt::trace {
bool enabled();
// Append {"t_us":..,"role":..,"sid":..,"ev":..} to $TUNNEL_TRACE.
void event(const char* role, uint32_t stream_id, const char* ev);
// The same with a time taken earlier (CLOCK_MONOTONIC us), e.g. a
// connection's accept stamped once its first request has a stream id.
void event_at(const char* role, uint32_t stream_id, const char* ev, uint64_t t_us);
void flush();  // buffered mode (TUNNEL_TRACE_BUFFERED=1): write out what is held
}  // namespace p2pt::trace
