// Per-thread CPU pinning inside the process's CPU set (TUNNEL_PIN_THREADS=1).
//
// A thread that migrates between CPUs in the middle of a large loopback TCP
// write leaves segments of one connection on two CPUs' receive backlogs; the
// second CPU's softirq can deliver its segments first. On the MI355X host the
// tunneled leg of the 64 x 1 MB echo showed exactly that (TCPOFOQueue 33-74,
// TCPSACKReorder 19-28, DSACK-undone fast retransmits per run; the direct leg
// none), and each spurious recovery shrinks that connection's window. With
// the switch on, the association thread takes the set's first CPU and every
// other registered thread (workers, lanes, socket reader) one of the rest,
// round robin, so none of them migrates. Default: on when the process was
// given its CPUs (--cpu-affinity; A/B on the host: +18-22 % at 1200 MTU,
// +18 % jumbo on the echo, profiles/r04/pt20), off otherwise (a process
// that may run anywhere is not packed onto the machine's first CPUs).
#pragma once

namespace p2pt::affinity {

// The default when TUNNEL_PIN_THREADS is not set (called before any thread starts).
void set_default(bool on);
bool enabled();
// Pins the calling thread (the association thread: the set's first CPU).
void pin_this_thread(bool assoc);
// CPUs of the process's set as it was before any thread pinned itself (the
// calling thread's set when nothing was pinned).
long process_cpu_count();

}  // namespace p2pt::affinity
