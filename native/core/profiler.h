// In-process sampling CPU profiler for the tunnel binaries (the
// reference has no profiler hooks at all; this container has no `perf`).
//
// TUNNEL_PROFILE=<path>[@HZ] ("%p" = pid) arms ITIMER_PROF at HZ (default 2000)
// (process CPU time: whichever thread runs gets sampled). The SIGPROF handler records the interrupted PC, the
// word at the stack pointer (the return address when a frameless leaf such as
// memcpy or an AES routine was interrupted) and up to kDepth frame-pointer
// links (our code is built with -fno-omit-frame-pointer), into a fixed,
// lock-free table — no allocation in the handler. At exit the table is written
// as text: one line per distinct stack, addresses resolved to
// "module+0xoffset" with dladdr. scripts/profile_report.py symbolises it with
// llvm-symbolizer and prints self/inclusive tables.
#pragma once

namespace p2pt::profiler {

// Starts sampling when TUNNEL_PROFILE is set; returns whether it did.
bool start_from_env();
// Writes the report now (also registered with atexit).
void dump();
// Records the calling thread's stack bounds so its samples get a frame-
// pointer walk (worker threads call this when they start).
// `tag` labels the thread's samples in the dump ("T<tag>"; 0 = main).
void register_thread(int tag);

// TUNNEL_THREAD_TIMELINE=<path> ("%p" = pid): every 2 ms a sampler thread
// reads each registered thread's CPU clock; at exit it writes, per thread, how
// many 2 ms intervals it spent at each utilisation level (JSON). A pipeline
// stage that saturates only in one phase of a workload (the upload half of a
// bulk echo step, say) shows as intervals at >= 90 % although its average is
// far lower. Call after start_from_env() on the main thread.
bool start_timeline_from_env();

}  // namespace p2pt::profiler
