// Per-thread CPU pinning inside the process's CPU set (TUNNEL_PIN_THREADS=1).
//
// A thread that migrates between CPUs in the middle of a large loopback TCP
// write leaves segments of one connection on two CPUs' receive backlogs; the
// second CPU's softirq can deliver its segments first. On the MI355X host the
// tunneled leg of the 64 x 1 MB echo showed exactly that (TCPOFOQueue 33-74,
// TCPSACKReorder 19-28, DSACK-undone fast retransmits per run; the direct leg
// none), and each spurious recovery shrinks that connection's window. With
// the switch on, every tunnel thread is pinned to one CPU of the set (see
// pin_this_thread for the layout), so none of them migrates. Default: on when the process was
// given its CPUs (--cpu-affinity; A/B on the host: +18-22 % at 1200 MTU,
// +18 % jumbo on the echo, profiles/r04/pt20), off otherwise (a process
// that may run anywhere is not packed onto the machine's first CPUs).
#pragma once

namespace p2pt::affinity {

// The default when TUNNEL_PIN_THREADS is not set (called before any thread starts).
void set_default(bool on);
bool enabled();
// Pins the calling thread by its role (profiler tags): 0 the association
// thread, 1.. HTTP workers, 90 TX seal lane, 91 RX lane, 92 socket reader,
// 93 TX send lane, 94 second sealer, 95 / 96 the socket reader's record-
// opening lanes. In the set's order: the association thread, the workers,
// the seal and send stages, the socket reader, the RX lane (with the second
// sealer), then the two open lanes — each on a CPU of its own from 8 CPUs up
// (the workers get n - 7), on the RX lane's CPU below that (with n - 5
// workers from 6 CPUs, one on 5), where only one open lane runs
// (open_lane_count). With fewer than 5 CPUs: round robin.
void pin_this_thread(int tag);
// Open lanes the socket reader should start (of `want`): 1 when pinned on a
// set too small to give them CPUs of their own, else `want`.
int open_lane_count(int want);
// CPUs of the process's set as it was before any thread pinned itself (the
// calling thread's set when nothing was pinned).
long process_cpu_count();

}  // namespace p2pt::affinity
