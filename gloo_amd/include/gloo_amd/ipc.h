// ipc.h — device memory shared between rank processes over HIP IPC.
//
// Why this exists ("IPC imports"): on ROCm 7 / MI355X an import
// of a handle that is byte-identical to an earlier one — the exporter freed a
// block and its next block of the same size came back at the same address,
// and a HIP IPC handle encodes (address, pid, size) — was handed the EARLIER
// import's mapping, i.e. the freed block's pages, after the importer had
// closed it (profiles/round3/r3b_*: every read path through the mapping, the
// runtime's copy and the GPU's own loads alike, showed the old contents).
// Freeing and re-exporting a block is therefore never safe while any peer
// process lives.  So:
//
//   Exporter side: every block that another process maps is a Slab from a
//   process-wide pool.  A slab is allocated and exported ONCE; an executor
//   that no longer needs it returns it to the pool, and the next executor
//   needing that size class on that device reuses it.  A trim frees the
//   free-listed slabs and RETIRES their addresses: no later slab of this
//   process is ever exported at a retired address (acquire parks such an
//   allocation and allocates again).  So an address a peer has imported
//   always maps the same pages, and a byte-identical handle always means
//   the same memory, with or without trims.  Trims are collective
//   (trimCollective in context.h): every rank first closes the mappings no
//   executor holds, then, after a barrier, frees its unused slabs — ROCm 7
//   fails the next export of memory allocated over a slab freed while a peer
//   still mapped it.  They run when a rank's pool would pass
//   GLOO_AMD_IPC_POOL_MAX (default 16 GiB): at an executor's construction
//   (before its slabs are acquired) and at a context's destruction.
//   Size classes are powers of two of 2 MiB granules up to 1 GiB, then
//   multiples of 256 MiB (a 1.5 GiB arena must not become a 2 GiB slab:
//   importing blocks of 2 GiB or more hangs on this platform, so the
//   executor refuses arenas that large between processes), so the pool holds
//   at most about twice the largest set of simultaneously live arenas.
//
//   Importer side: a mapping is opened once per (exporter pid, exporter
//   incarnation, exporter address) and kept, counted by the executors that
//   hold it; a trim closes the mappings no executor holds (a later import
//   of the same slab opens it afresh, which is safe because the exporter
//   never re-exports that address for other pages).
//   The incarnation (a random word per process) tells a new process that
//   reuses a dead one's pid apart; its old mappings are closed first.
//
// Callers still verify each import (executor.cc writes a nonce at the slab's
// start and every importer reads it back): a mismatch is a hard error.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace gloo_amd {
namespace ipc {

struct Slab {
  char* ptr = nullptr;
  size_t bytes = 0;  // the size class (>= what was asked for)
  int device = -1;
  bool fine = false;  // fine-grained (cross-device coherent) memory
  hipIpcMemHandle_t handle;
};

// A random word fixed for the life of this process.
uint64_t incarnation();

// A slab of at least `bytes` on `device` (fine-grained or not), exported.
Slab* acquire(int device, size_t bytes, bool fine);
// Back to the pool (never hipFree'd).  The caller has made sure no peer
// still writes into it (the executor's tear-down barrier).
void release(Slab* s);

// The mapping of a peer process's slab (opened once, kept).
void* import(int pid, uint64_t incarnation, uint64_t ptr, size_t bytes, const hipIpcMemHandle_t& handle);
// Drops an executor's hold on a mapping (kept until a trim).
// GLOO_AMD_IPC_POOL=0 (diagnosis only) restores the behaviour the pool
// replaced: release() frees the slab at once and unimport() closes the
// mapping (tools/ipc_bisect.sh reproduces the stale import with it).
void unimport(void* mapped);
bool poolEnabled();
// The two halves of a trim (above): close this process's mappings no
// executor holds; free (and retire) its free-listed slabs.
void closeUnusedImports();
void freeUnusedSlabs();
// Whether the pool holds free slabs and would pass its ceiling with `more`
// bytes of new slabs.
bool overCeiling(size_t more);
// Both halves at once, for a process whose peers are gone (gloo_hip_ipc_trim).
inline void trim() {
  closeUnusedImports();
  freeUnusedSlabs();
}

struct Stats {
  size_t slabs = 0, slabBytes = 0, free = 0, imports = 0, opens = 0;
  size_t trims = 0, trimmedBytes = 0, closes = 0, retired = 0, parked = 0, max = 0;
};
Stats stats();

}  // namespace ipc
}  // namespace gloo_amd
