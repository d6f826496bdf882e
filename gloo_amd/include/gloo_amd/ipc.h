// ipc.h — device memory shared between rank processes (inbox arenas,
// mailboxes, transport landing slabs).
//
// The mechanism is HIP's virtual memory management with dma-buf file
// descriptors (VMM); the rounds 3-4 hipIpc pool remains behind
// GLOO_AMD_IPC=hipipc.  Every rank of a collective must use the same one,
// and the executor refuses a mix on every rank.
//
// VMM.  A slab is a hipMemCreate block exported once as a dma-buf fd.
//   * Any size maps: 2.5 GiB end to end in ~20 ms (tools/vmm_probe,
//     profiles/round5/r5b_vmm_fresh_va.jsonl), where a hipIpc import of 2 GiB
//     or more hangs (profiles/round3/r3t_*, r3u_*).
//   * A virtual range is never mapped twice, and never freed: a new block
//     mapped where an earlier mapping lived showed the earlier block's pages,
//     then faulted (r5a_vmm_same_va_*, r5b_vmm_same_va.err), and so did a
//     range freed with hipMemAddressFree and handed out again by the next
//     reserve (r5j_vmm_sys_freeva_uncached.jsonl).  Since HIP returns a
//     block's memory only when its range is freed (tools/vmm_leak.py,
//     r5i_*), slabs and imports are never released: they are reused by
//     size class (powers of two of 2 MiB up to 1 GiB, then multiples of
//     256 MiB), which bounds the pool by the classes a process uses.
//   * Peers obtain a slab's fd from its owner's fd server: a thread on an
//     abstract Unix socket named by (pid, incarnation) that answers a slab id
//     with the fd (SCM_RIGHTS), to processes of the same user only.
//   * hipMemImportFromShareableHandle takes the fd by value on HIP 7.2 (the
//     system ROCm) and by address on HIP 7.0.51831 (the runtime PyTorch
//     2.10+rocm7.0 bundles and loads in place of the system one), which
//     crashes on the value (r5j_vmm_torch_*): chosen by runtime version.
//
// hipIpc (GLOO_AMD_IPC=hipipc).  A slab is a hipMalloc / fine-grained block
//   exported with hipIpcGetMemHandle, ONCE: a freed block re-exported at the
//   same address was imported as the old pages (profiles/round3/r3b_*), so
//   slabs are reused, and a trim's freed slabs retire their address ranges (a
//   block the runtime hands out inside one is parked, never exported).
//   Imports of 2 GiB and more hang, so slabs stay below 2^31 bytes and the
//   executor refuses larger cross-process arenas.  Under heavy churn the
//   runtime can keep handing out retired addresses until acquire gives up
//   after 64 tries (profiles/round5/r5c_pytest_churn_hipipc.log).
//   Trims (when the pool would pass GLOO_AMD_IPC_POOL_MAX, default 16 GiB)
//   are collective: every rank first closes the mappings no executor holds,
//   then frees its free slabs.
//
// Both: an executor that no longer needs a slab returns it to the pool, and
// the next executor of that size class on that device reuses it (its peers'
// mappings too).  Imports are kept per (exporter pid, incarnation, slab) and
// counted per executor; the incarnation (a random word per process) tells a
// new process that reuses a dead one's pid apart.  Callers verify each
// import (the executor writes a nonce at the slab's start and every importer
// reads it back): a mismatch is a hard error.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace gloo_amd {
namespace ipc {

// The mechanism of this process: true = VMM (see above).
bool vmm();
// hipRuntimeGetVersion() of the loaded HIP runtime (e.g. 70226015 for 7.2).
int runtimeVersion();
// Largest slab the mechanism can share (hipIpc: below 2 GiB; VMM: no limit).
size_t maxSlabBytes();

struct Slab {
  char* ptr = nullptr;   // this process's mapping
  size_t bytes = 0;      // the size class (>= what was asked for)
  int device = -1;
  bool fine = false;     // cross-device coherent memory (VMM: uncached; hipIpc: fine-grained)
  uint64_t id = 0;       // names the slab to peers
  hipMemGenericAllocationHandle_t handle = nullptr;  // VMM
  int fd = -1;                                       // VMM: the exported dma-buf
  hipIpcMemHandle_t ipcHandle;                       // hipIpc
};

// What a peer publishes about one of its slabs.
struct Remote {
  int pid = 0;
  uint64_t incarnation = 0;
  uint64_t id = 0;                 // VMM
  uint64_t ptr = 0;                // hipIpc: the exporter's address
  hipIpcMemHandle_t ipcHandle;     // hipIpc
};
Remote describe(const Slab& s);

// A random word fixed for the life of this process.
uint64_t incarnation();

// A slab of at least `bytes` on `device`, exported (VMM: starts this
// process's fd server on first use).
Slab* acquire(int device, size_t bytes, bool fine);
// Back to the pool.  The caller has made sure no peer still writes into it
// (the executor's tear-down barrier).
void release(Slab* s);

// The mapping of a peer process's slab, accessible from `device` (opened
// once, kept).  `bytes`: what the caller will touch.
void* import(const Remote& r, size_t bytes, int device);
// Drops an executor's hold on a mapping (kept until a trim).
void unimport(void* mapped);
// The two halves of a trim (above).
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
  size_t vmm = 0;  // 1: the VMM mechanism
};
Stats stats();

}  // namespace ipc
}  // namespace gloo_amd
