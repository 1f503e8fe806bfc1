// oracle/ref_executor_harness.cc -- TEST INFRASTRUCTURE ONLY.
//
// Compiles the reference executor's own translation unit
// (executor/executor_linux.cc, which pulls in executor.h) exactly as it lies
// under the reference checkout, with its `main` renamed so the unit can be a
// shared library, and exposes the reference's static hash()/dedup()
// (executor/executor.h:497-526) plus a driver that replays the signal loop of
// handle_completion (executor/executor.h:389-401) over synthetic traces.
// Nothing is stubbed: every symbol comes from the reference sources.
// Built by oracle/Makefile into oracle/_ref/ (git-ignored).
#define main syz_executor_main
#include "executor_linux.cc"
#undef main

extern "C" uint32_t ref_exec_hash(uint32_t a) { return hash(a); }
extern "C" void ref_exec_reset(void) { memset(dedup_table, 0, sizeof(dedup_table)); }
extern "C" int ref_exec_dedup(uint32_t sig) { return dedup(sig) ? 1 : 0; }

// Signal of one call, appended to out; uses the reference hash/dedup and the
// shared global dedup_table (reset per program by the caller, like fork()).
extern "C" uint32_t ref_exec_call_signal(const uint32_t* pcs, uint32_t n, uint32_t* out)
{
	uint32_t nsig = 0;
	uint32_t prev = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint32_t pc = pcs[i];
		uint32_t sig = pc ^ prev;
		prev = hash(pc);
		if (dedup(sig))
			continue;
		out[nsig++] = sig;
	}
	return nsig;
}
