// ipc.h — device memory shared between rank processes (inbox arenas,
// mailboxes, transport landing slabs).
//
// The mechanism is HIP's virtual memory management with dma-buf file
// descriptors (VMM).  A slab is a hipMemCreate block exported once as a
// dma-buf fd.
//   * Any size maps: 2.5 GiB end to end in ~20 ms (tools/vmm_probe,
//     profiles/round5/r5b_vmm_fresh_va.jsonl), where a hipIpc import of 2 GiB
//     or more hangs (profiles/round3/r3t_*, r3u_*).
//   * A virtual range is never mapped twice, and never freed: a new block
//     mapped where an earlier mapping lived showed the earlier block's pages,
//     then faulted (r5a_vmm_same_va_*, r5b_vmm_same_va.err), and so did a
//     range freed with hipMemAddressFree and handed out again by the next
//     reserve (r5j_vmm_sys_freeva_uncached.jsonl).  Since HIP returns a
//     block's memory only when its range is freed (tools/vmm_leak.py,
//     r5i_*), slabs are never released while the process lives: they are
//     created in size classes (powers of two of 2 MiB up to 1 GiB, then
//     multiples of 256 MiB) and a request is served from the smallest idle
//     slab that holds it (best fit), so a process never holds more than
//     one slab per class it used at once, and a class never used before is
//     served from a larger idle slab when there is one.  When hipMemCreate
//     runs out of memory the error names the pool's idle bytes.  An import
//     nobody holds is unmapped once its exporter has exited.
//   * Peers obtain a slab's fd from its owner's fd server: a thread on an
//     abstract Unix socket named by (pid, incarnation) that answers a slab id
//     with the fd (SCM_RIGHTS), to processes of the same user only.
//   * hipMemImportFromShareableHandle takes the fd by value on HIP 7.2 (the
//     system ROCm) and by address on HIP 7.0.51831 (the runtime PyTorch
//     2.10+rocm7.0 bundles and loads in place of the system one), which
//     crashes on the value (r5j_vmm_torch_*): chosen by runtime version.
// Rounds 3-4 shared hipMalloc blocks through hipIpc handles instead; that
// pool (trims, retired address ranges, parked blocks, a 1.75 GiB cap) is
// gone (DESIGN.md "Cross-process memory").
//
// An executor that no longer needs a slab returns it to the pool, and the
// next executor on that device whose request it holds reuses it (its peers'
// mappings too).  Imports are kept per (exporter pid, slab id) and counted
// per executor; the incarnation (a random word per process) tells a new
// process that reuses a dead one's pid apart.  Callers verify each import
// (the executor writes a nonce at the slab's start and every importer reads
// it back): a mismatch is a hard error.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace gloo_amd {
namespace ipc {

// hipRuntimeGetVersion() of the loaded HIP runtime (e.g. 70226015 for 7.2).
int runtimeVersion();

struct Slab {
  char* ptr = nullptr;   // this process's mapping
  size_t bytes = 0;      // the size class (>= what was asked for)
  int device = -1;
  bool fine = false;     // uncached memory: what a peer writes is never behind a stale line
  uint64_t id = 0;       // names the slab to peers
  hipMemGenericAllocationHandle_t handle = nullptr;
  int fd = -1;           // the exported dma-buf
  uint64_t devices = 0;  // bit d: device d of this process may access the mapping
};

// What a peer publishes about one of its slabs.
struct Remote {
  int pid = 0;
  uint64_t incarnation = 0;
  uint64_t id = 0;
};
Remote describe(const Slab& s);

// A random word fixed for the life of this process.
uint64_t incarnation();

// A slab of at least `bytes` on `device`, exported (starts this process's fd
// server on first use).
Slab* acquire(int device, size_t bytes, bool fine);
// Back to the pool.  The caller has made sure no peer still writes into it
// (the executor's tear-down barrier).
void release(Slab* s);

// The mapping of a peer process's slab, accessible from `device` (mapped
// once, kept).  `bytes`: what the caller will touch.
void* import(const Remote& r, size_t bytes, int device);
// Drops an executor's hold on a mapping (the mapping stays for reuse).
void unimport(void* mapped);
// A VMM mapping is accessible only from the devices it was granted to (a
// peer-access enable does not cover it): lets `device` of this process read
// and write one of the pool's slabs or imports, given its mapped address (a
// rank of this process on another GPU sending into a slab; no-op when the
// address is not the pool's).
void grantAccess(void* mapped, int device);

// A range of a caller's device allocation (hipMalloc memory, not a pool
// slab) shared with peer processes: exported as a dma-buf of its allocation
// through the HSA runtime the HIP runtime loaded
// (hsa_amd_portable_export_dmabuf), served by this process's fd server under
// an id, and imported by a peer with hipMemImportFromShareableHandle into a
// virtual range never mapped before (tools/dmabuf_probe.cc,
// profiles/round6/r6d/dmabuf_probe.jsonl: reads and writes both ways, and a
// block freed and allocated again at the same address exports as the NEW
// block).  This replaces the hipIpc handles of rounds 1-5.
struct RangeExport {
  uint64_t id = 0;      // names the export to peers (fd server)
  uint64_t offset = 0;  // of the range within its dma-buf
  uint64_t bytes = 0;
};
// false: the runtime cannot export this memory (the caller falls back).
bool exportRange(const void* ptr, size_t bytes, RangeExport* out);
void unexportRange(const RangeExport& e);
struct RangeImport {
  char* ptr = nullptr;  // the peer's range, mapped here
  void* va = nullptr;   // the mapping (reserved for good: ipc.h "never mapped twice")
  size_t vaBytes = 0;
  hipMemGenericAllocationHandle_t handle = nullptr;
};
// Maps a peer's exported range (r.id = the export's id) for `device`.
RangeImport importRange(const Remote& r, uint64_t offset, size_t bytes, int device);
void unimportRange(RangeImport* m);

struct Stats {
  size_t slabs = 0, slabBytes = 0, free = 0, imports = 0, opens = 0;
  size_t dropped = 0;  // mappings of exited processes (their pid reused) unmapped
};
Stats stats();

}  // namespace ipc
}  // namespace gloo_amd
