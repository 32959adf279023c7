/* reacher_comm.h -- the one data-path collective of the sharded rollout (libreacher.so):
 * an in-place SUM all-reduce of a flat f32 gradient over RCCL (xGMI), issued on the
 * trainer's own HIP stream.
 *
 * Why a communicator of our own beside torch.distributed: torch's collective runs on an
 * internal stream, so every step pays two cross-stream event waits plus ~19 us of host
 * dispatch per call (measured on one MI355X with a world-size-1 group, 262,144 envs: the
 * torch path costs a c4 step 117 -> 126 us before any exchange happens;
 * scripts/allreduce_overhead.py).  Here the all-reduce is one more launch on the stream that
 * already holds the rollout and the Adam kernel, and rdd_step() issues the whole sharded
 * step (rollout, reduce, all-reduce, Adam) from one host call.
 *
 * The reference has no multi-GPU path in src/distilation; its only collective is MpiAdam's
 * Allreduce(SUM) of the flat gradient (reference backup/student_rollout.py:658-659,709) --
 * this is that exchange, once per optimiser step.
 *
 * RCCL is resolved at run time (dlopen of librccl.so.1, reusing the copy torch loaded), so
 * the library loads on hosts without RCCL; rd_comm_* then fail with RD_EINVAL and a message.
 * Usage (one process per GPU): every rank calls rd_comm_probe() and the ranks agree on the
 * result (e.g. an all-reduce over the torch.distributed group), so a rank that cannot take
 * part stops everyone before any RCCL collective starts; rank 0 calls rd_comm_unique_id()
 * and broadcasts the 128 bytes; every rank calls rd_comm_create() with them; bind with
 * rdd_bind_comm() (reacher_distill.h).  The communicator is non-blocking underneath: its
 * creation (and a first collective's connection setup) is awaited with a deadline, and a
 * rank whose peers do not arrive within timeout_s aborts the communicator and returns an
 * error instead of hanging.  Conventions as in reacher.h.
 */
#ifndef REACHER_COMM_H
#define REACHER_COMM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RD_COMM_ID_BYTES 128

typedef struct rd_comm rd_comm;

/* A fresh RCCL unique id (rank 0 only); id: host buffer of RD_COMM_ID_BYTES. */
int rd_comm_unique_id(uint8_t* id);

/* 0 iff this rank can join: RCCL resolvable and HIP device `device` selectable. */
int rd_comm_probe(int device);

/* Collective over all ranks: an RCCL communicator of nranks ranks on HIP device `device`;
 * fails (communicator aborted) if the other ranks have not joined within timeout_s. */
int rd_comm_create(rd_comm** out, const uint8_t* id, int nranks, int rank, int device, double timeout_s);

/* In-place SUM all-reduce of n floats of device memory, asynchronous on hip_stream. */
int rd_comm_allreduce_f32(rd_comm* c, float* buf, int64_t n, void* hip_stream);

int rd_comm_nranks(const rd_comm* c);
/* RCCL's own view of the communicator: ncclCommCount, ncclCommUserRank, ncclCommCuDevice
 * (from_rccl = 1); for an xGMI communicator (no RCCL object) the values it was created with
 * (from_rccl = 0).  Host-synchronous. */
int rd_comm_query(rd_comm* c, int* count, int* user_rank, int* device, int* from_rccl);
int rd_comm_destroy(rd_comm* c);

/* The same exchange without RCCL: a one-shot push over xGMI (rd_xgmi.hip).  Each rank
 * allocates an exchange buffer of uncached device memory (2 x RD_XG ranks x `cap` floats +
 * flags) and exports it: rd_xcomm_create() writes this rank's RD_XCOMM_HANDLE_BYTES IPC handle
 * to `handle`; the ranks all-gather the handles (e.g. over the torch.distributed group) and
 * every rank calls rd_xcomm_connect() with the nranks handles in rank order, which maps every
 * peer's buffer.  rd_comm_allreduce_f32() on such a communicator is ONE kernel per exchange:
 * each rank writes its n <= cap floats into its slot of every rank's buffer (one block per
 * destination, all xGMI links at once), raises a flag there, waits for every flag in its own
 * buffer and sums the slots in rank order -- so every rank gets bitwise the same sum.  At most
 * 8 ranks (one node).
 * Failure: a wait that does not see a peer within timeout_s (wall clock) FAILS the
 * communicator on every rank: the kernel leaves the buffer unsummed, raises this rank's error
 * word and poisons every peer's buffer, so a peer that arrives later fails its exchange too
 * instead of completing it alone.  The blocks of one exchange agree on one outcome per rank
 * (each posts its verdict on a device counter; the decision is taken once all are in), so a
 * rank's gradient is either fully summed or untouched.  A trainer with the communicator bound
 * skips the Adam update of a failed exchange (no replica applies a partial sum) and its next
 * rdd_step / rdd_allreduce_grad / counter read returns RD_ECOMM; rd_comm_check() returns
 * RD_ECOMM without synchronising.  A failed communicator fails every later exchange: destroy
 * it.  Across ranks the outcome is not atomic: a peer whose last flag lands within the final
 * poll before this rank's deadline can have summed and stepped while this rank skipped, so
 * after RD_ECOMM the student parameters AND the Adam state must be re-broadcast from one rank
 * before training resumes on a new communicator (the replica checksum,
 * DistillTrainer.replicas_identical, detects a divergence).  timeout_s bounds rank-local host
 * work between two exchanges too: a rank held longer than that (checkpoint I/O, evaluation on
 * rank 0 only) fails the communicator for good, so size it above any such pause (dist.XgmiComm
 * defaults to 600 s; torch/RCCL collectives default to 30 min).  The reference's exchange it
 * replaces: MpiAdam's Allreduce(SUM) (backup/student_rollout.py:658-659,709). */
#define RD_XCOMM_HANDLE_BYTES 64
int rd_xcomm_create(rd_comm** out, int nranks, int rank, int device, int64_t cap, double timeout_s, uint8_t* handle);
int rd_xcomm_connect(rd_comm* c, const uint8_t* handles);
int rd_comm_check(rd_comm* c);

#ifdef __cplusplus
}
#endif
#endif
