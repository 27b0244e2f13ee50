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
void flush();  // write out what is held (also done at exit)

// Transport hops of a traced frame (this thread's current datagrams):
// the receive side records when the kernel queued the datagram (SO_TIMESTAMPNS,
// converted to CLOCK_MONOTONIC), when a thread read it, and when the
// association thread took it up; rx_stamps() writes them for a stream as
// udp_kernel / udp_read / rx_assoc. The send side queues a stream with
// mark_tx() and the datagram flush that carries it stamps udp_tx (tx_done(),
// called just before the flush's first send syscall).
void set_rx(uint64_t kernel_us, uint64_t read_us, uint64_t assoc_us);
void rx_stamps(const char* role, uint32_t stream_id);
void mark_tx(const char* role, uint32_t stream_id);
void tx_done();
// Monotonic microseconds of a SCM_TIMESTAMPNS (CLOCK_REALTIME) cmsg in the
// message, 0 if none.
uint64_t kernel_rx_us(const void* msghdr);
}  // namespace p2pt::trace
