// ipc.h — device memory shared between rank processes (inbox arenas and
// mailboxes), through HIP's virtual memory management with dma-buf file
// descriptors.
//
// Why this form ("Cross-process memory"):
//   * hipIpcGetMemHandle / hipIpcOpenMemHandle, the route of rounds 1-4,
//     hangs on imports of 2 GiB and more on ROCm 7 / MI355X, and an import of
//     a byte-identical handle (a freed block re-exported at the same address)
//     was handed the old pages (profiles/round3/r3b_*, r3t_*, r3u_*).
//   * A VMM block (hipMemCreate, POSIX-fd handle type) exported with
//     hipMemExportToShareableHandle and imported with
//     hipMemImportFromShareableHandle maps at any size — 2.5 GiB end to end in
//     22 ms (tools/vmm_probe, profiles/round5/r5b_vmm_fresh_va.jsonl).
//   * But a virtual range must never be mapped twice: a new block mapped at a
//     virtual address an earlier mapping used showed the earlier block's
//     pages, and then faulted (r5a_vmm_same_va_*, r5b_vmm_same_va.err) —
//     translations of the old mapping survive the unmap.  With every mapping
//     at a range never used before, the same churn — free, re-allocate,
//     re-import, graph copies into the mapping — is exact (r5b_vmm_fresh_va).
// So:
//   Exporter side: every block another process maps is a Slab of a
//   process-wide pool: a VMM allocation mapped at a fresh virtual range,
//   exported once as a dma-buf fd that the process keeps open.  Peers obtain
//   that fd from this process's fd server — a thread on an abstract Unix
//   socket named by (pid, incarnation) that answers "slab id" with the fd
//   (SCM_RIGHTS), to processes of the same user only.  An executor that no
//   longer needs a slab returns it to the pool; the next executor of that
//   size class on that device reuses it (its peers' mappings too).  A trim
//   (when the pool would pass GLOO_AMD_IPC_POOL_MAX, default 16 GiB) unmaps
//   and releases the free slabs; their virtual ranges stay reserved and are
//   never mapped again (retired).  Trims are collective (every rank first
//   closes the mappings no executor holds, then frees), so no slab is
//   released while a peer still maps it.
//   Importer side: a mapping is opened once per (exporter pid, incarnation,
//   slab id) at a fresh virtual range and kept, counted by the executors that
//   hold it; a trim closes the ones no executor holds (unmap, release; the
//   range is retired).  The incarnation (a random word per process) tells a
//   new process that reuses a dead one's pid apart.
//   Size classes are powers of two of 2 MiB up to 1 GiB, then multiples of
//   256 MiB; there is no upper bound.
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
  char* ptr = nullptr;   // this process's mapping
  size_t bytes = 0;      // the size class (>= what was asked for)
  int device = -1;
  bool fine = false;     // uncached (cross-device coherent) memory
  uint64_t id = 0;       // names the slab to peers (the fd server)
  hipMemGenericAllocationHandle_t handle = nullptr;
  int fd = -1;           // the exported dma-buf
};

// A random word fixed for the life of this process.
uint64_t incarnation();

// A slab of at least `bytes` on `device` (uncached or not), exported; starts
// this process's fd server on first use.
Slab* acquire(int device, size_t bytes, bool fine);
// Back to the pool (not released).  The caller has made sure no peer still
// writes into it (the executor's tear-down barrier).
void release(Slab* s);

// The mapping of a peer process's slab `id`, accessible from `device`
// (opened once, kept).  `bytes`: what the caller will touch.
void* import(int pid, uint64_t incarnation, uint64_t id, size_t bytes, int device);
// Drops an executor's hold on a mapping (kept until a trim).
void unimport(void* mapped);
// The two halves of a trim (above): close this process's mappings no
// executor holds; release its free-listed slabs.
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
  size_t trims = 0, trimmedBytes = 0, closes = 0, retired = 0, retiredBytes = 0, max = 0;
};
Stats stats();

}  // namespace ipc
}  // namespace gloo_amd
