/*
 * dcol.h — C-ABI of the MI355X-native batched differentiable-proximity engine.
 *
 * Drop-in boundary for the reference's proximity hot path
 * (CogSP/DCOL-trajectory-optimization):
 *
 *   reference                                                 replaced by
 *   ------------------------------------------------------   ---------------------------------
 *   primitive objects consumed by problem_matrices()          dcol_table_create()
 *     primitives/misc_primitive_constructor.py:4-88             (static shape table, uploaded
 *     primitives/problem_matrices.py:255-364                     once to HBM)
 *   proximity_mrp(prim1, prim2, pdip_tol) -> (alpha, x[:3])   dcol_plan_run(flags=CONTACT)
 *     proximity/proximity.py:6-54                             dcol_prox_batch_host()
 *                                                             dcol_prox_pair() (one pair)
 *   proximity_gradient(prim1, prim2, pdip_tol)                dcol_plan_run(flags=GRAD_FD)
 *     -> (alpha, d_alpha/d[r1,p1,r2,p2])                      dcol_prox_batch_host()
 *                                                             dcol_prox_pair() (one pair)
 *     proximity/proximity_gradient.py:91-138
 *   combine_problem_matrices() + solve_lp_pdip()              inside the device kernel
 *     primitives/combine_problem_matrices.py:3-70,
 *     proximity/pdip.py:291-470, proximity/NT/NT_scaling.py
 *
 * One call handles a whole batch of (knot x primitive-pair) problems.  All arithmetic is
 * IEEE FP64.  Plain pointers and sizes only; no torch types.  Error behaviour: every entry
 * point returns an int (DCOL_SUCCESS or a negative DCOL_ERR_*); per-pair solver outcomes
 * are reported in a status[] array (enum dcol_status), which the Python shim maps back to
 * the reference's exception types (bare Exception at 50 iterations, pdip.py:470;
 * ValueError for unsupported pairs, combine_problem_matrices.py:70; LinAlgError for a
 * non-PD normal matrix, pdip.py:317/:434).
 */
#ifndef DCOL_H
#define DCOL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCOL_ABI_VERSION 4   /* 2: 14-slot multi-GPU record (status / iters as an int32 pair);
                                3: DCOL_NO_GATHER + dcol_comm_all_gather, dcol_table_pair_plans,
                                   dcol_table_pair_stats;
                                4: dcol_plan_num_streams, dcol_plan_launch_form, dcol_shutdown,
                                   dcol_table_stop_pair_server, dcol_table_pair_server_running,
                                   dcol_debug_pair_stamps */

/* Primitive types (misc_primitive_constructor.py:4-88). */
enum dcol_shape_type {
    DCOL_POLYTOPE = 0, /* A (nh x 3), b (nh)          PolytopeMRP  */
    DCOL_SPHERE = 1,   /* R                           SphereMRP    */
    DCOL_CONE = 2,     /* H, beta (half angle, rad)   ConeMRP      */
    DCOL_CAPSULE = 3,  /* R, L                        CapsuleMRP   */
    DCOL_CYLINDER = 4, /* R, L                        CylinderMRP  */
    DCOL_POLYGON = 5   /* A (nh x 2), b (nh), R       PolygonMRP   */
};

/* Per-pair outcome. */
enum dcol_status {
    DCOL_OK = 0,
    DCOL_MAXITER = 1,     /* no convergence within max_iter (reference: 50, pdip.py:408)  */
    DCOL_UNSUPPORTED = 2, /* both primitives have extra columns (combine case 4)          */
    DCOL_NOT_PD = 3,      /* Cholesky of G'G or of the NT normal matrix failed            */
    DCOL_NONFINITE = 4,   /* a non-finite value reached a factorisation                   */
    DCOL_TOO_LARGE = 5    /* more orthant rows than the engine's row capacity (128)       */
};

/* dcol_plan_run / dcol_prox_batch_host flags. */
enum dcol_flags {
    DCOL_GRAD_FD = 1,       /* d alpha / d[r1,p1,r2,p2] by 2-point forward differences of
                               z'(G(theta)x - h(theta)), step sqrt(eps) (reference mode,
                               proximity_gradient.py:50-88)                               */
    DCOL_GRAD_ENVELOPE = 2, /* the same gradient in closed form (envelope theorem)       */
    DCOL_CONTACT = 4,       /* write x[0:3] (proximity.py:51-54)                          */
    DCOL_CASE4 = 8,         /* dcol_prox_batch_host only: solve case-4 pairs (see
                               DCOL_PLAN_CASE4) instead of reporting DCOL_UNSUPPORTED     */
    DCOL_GRAD_IMPLICIT = 16, /* implicit-function derivative of the returned iterate: the
                               KKT system linearised with the NT scaling at (x, s, z),
                               d alpha = e3' H^-1 (-dG'z - G'W^-2 (dG x - dh)) with H the
                               PDIP's normal matrix G'W^-2 G (same Cholesky routine), for
                               the 12 pose coordinates; equals the envelope gradient as
                               mu -> 0 (pdip.py:434; no reference counterpart)            */
    DCOL_NO_GATHER = 32     /* dcol_prox_batch_multi_gpu in place only: the solve and the
                               record writes of the call (this rank's rows of rec_all and
                               their NaN tail) WITHOUT the all-gather -- issue it with
                               dcol_comm_all_gather (e.g. on a stream of its own, so the
                               next step's solve overlaps it), or time the step without
                               its collective (comm = step - this, like for like)         */
};
#define DCOL_GRAD_ANY (DCOL_GRAD_FD | DCOL_GRAD_ENVELOPE | DCOL_GRAD_IMPLICIT)

/* dcol_plan_create_ex options. */
enum dcol_plan_options {
    DCOL_PLAN_CASE4 = 1, /* EXTENSION, not reference behaviour: pairs in which BOTH primitives
                           have extra columns (capsule/cylinder/polygon x capsule/cylinder/
                           polygon) — combine_problem_matrices.py:58-67 raises ValueError for
                           them — are assembled with primitive 2's extra columns placed after
                           primitive 1's (n = 4 + e1 + e2 <= 8) and solved by the same PDIP.
                           Without the option they get DCOL_UNSUPPORTED like the reference. */
    DCOL_PLAN_NO_FUSE = 2, /* always one launch per bucket.  By default a plan with several
                           buckets (kernel variants) whose pairs together fill less than one
                           wave per SIMD -- an ALTRO phase batch -- runs every bucket in ONE
                           fused launch (no stream fan-out); results are bitwise the same.  */
    DCOL_PLAN_SUSPEND = 4 /* large buckets with a suspend / resume kernel pair run as a main
                           launch in which each wave hands its last few iterating pairs to a
                           compact resume launch, instead of idling most of its lanes until
                           its slowest pair converges; results are bitwise the same.  The plan
                           then owns device scratch written by every run: do not run it on
                           two streams at once (one plan per stream).                       */
};

/* Return codes of every entry point. */
#define DCOL_SUCCESS 0
#define DCOL_ERR_ARG (-1)
#define DCOL_ERR_HIP (-2)
#define DCOL_ERR_NOMEM (-3)

/* One primitive (all fields read; unused ones ignored for the type). */
typedef struct dcol_shape_desc {
    int32_t type;        /* enum dcol_shape_type                                      */
    int32_t nh;          /* faces: rows of A (polytope / polygon), else 0             */
    const double* A;     /* row-major nh x 3 (polytope) or nh x 2 (polygon), or NULL  */
    const double* b;     /* nh, or NULL                                               */
    double R, L, H, beta;
    double r_offset[3];  /* body-frame position offset (problem_matrices.py:281)      */
    double Q_offset[9];  /* row-major 3x3 orientation offset (problem_matrices.py:282) */
} dcol_shape_desc;

typedef struct dcol_table dcol_table; /* device-resident shape table */
typedef struct dcol_plan dcol_plan;   /* static pairing -> kernel-variant buckets */

/* ---- library / errors --------------------------------------------------------------- */
int dcol_abi_version(void);
const char* dcol_status_string(int32_t status);
const char* dcol_last_error(void); /* thread-local message of the last failing call */
int dcol_device_count(int32_t* count);

/* ---- shape table ---------------------------------------------------------------------
 * Copies the descriptors (and A/b) into an immutable table in HBM of `device`.       */
int dcol_table_create(const dcol_shape_desc* shapes, int32_t n, int32_t device, dcol_table** out);
int dcol_table_destroy(dcol_table* table);
int dcol_table_size(const dcol_table* table, int32_t* n);
/* Problem size of a pair (m rows, n columns, number of SOC blocks); returns the pair's
 * static status (DCOL_OK, DCOL_UNSUPPORTED or DCOL_TOO_LARGE) in *status.            */
int dcol_pair_dims(const dcol_table* table, int32_t s1, int32_t s2, int32_t* m, int32_t* n,
                   int32_t* n_soc, int32_t* status);

/* ---- plans ---------------------------------------------------------------------------
 * A plan fixes the pairing (shape ids, HOST arrays of length B) and buckets the pairs by
 * kernel variant.  It is reusable for any poses: ALTRO evaluates the same
 * (knot x obstacle) pairing at every iteration (systems/<name>.py inequality_constraints_x). */
int dcol_plan_create(const dcol_table* table, int64_t B, const int32_t* shape1,
                     const int32_t* shape2, dcol_plan** out);
/* Same with options (enum dcol_plan_options); options = 0 is dcol_plan_create.         */
int dcol_plan_create_ex(const dcol_table* table, int64_t B, const int32_t* shape1,
                        const int32_t* shape2, int32_t options, dcol_plan** out);
int dcol_plan_destroy(dcol_plan* plan);
int dcol_plan_num_launches(const dcol_plan* plan, int32_t* n); /* kernel launches per run */
int dcol_plan_num_streams(const dcol_plan* plan, int32_t* n); /* streams a run spreads its launches over:
                                                                  the caller's + side streams (1 = caller's only) */
int dcol_plan_num_buckets(const dcol_plan* plan, int32_t* n);  /* variant buckets (incl. rejects) */
/* How a run launches its solve buckets: DCOL_FORM_BUCKETS one launch per bucket (over
 * dcol_plan_num_streams streams), DCOL_FORM_FUSED one fused launch (a small plan: latency
 * configurations), DCOL_FORM_PACKED one packed launch (a mid-size plan: throughput
 * configurations).                                                   */
enum dcol_plan_form { DCOL_FORM_BUCKETS = 0, DCOL_FORM_FUSED = 1, DCOL_FORM_PACKED = 2 };
int dcol_plan_launch_form(const dcol_plan* plan, int32_t* form);
/* Bucket i (0 <= i < dcol_plan_num_buckets) of a plan, for tests and tools: info[0] kind (0 a
 * solve bucket, 1 rejected pairs), [1] N (primal columns), [2] SOC blocks, [3] orthant-row
 * bucket OMAX, [4] lanes per pair the launch runs at, [5] extra-column slots of a row-
 * partitioned bucket (0: dense rows), [6] flags (1 padding-free, 2 ball-SOC rows, 4 cone-SOC
 * rows), [7] the status of a reject bucket (else 0); *pairs = its pair count.  No reference
 * counterpart (the plan is this library's own batching layer).                          */
int dcol_plan_bucket(const dcol_plan* plan, int32_t i, int32_t info[8], int64_t* pairs);
/* DCOL_PLAN_SUSPEND plans: pairs the last completed run handed to resume launches
 * (synchronous copy; call after the run's stream has been synchronised), else 0.       */
int dcol_plan_suspended(const dcol_plan* plan, int64_t* n);

/* Solve every pair of the plan.  All arrays are DEVICE pointers on the table's device,
 * structure-of-arrays:
 *   pose1, pose2 : [6][B]  (rows r_x r_y r_z p_x p_y p_z; p = MRP)
 *   alpha        : [B]      minimum uniform scaling (x[3])
 *   contact      : [3][B]   x[0:3]            (written if flags & DCOL_CONTACT, else may be NULL)
 *   grad         : [12][B]  d alpha/d[r1,p1,r2,p2] (if a GRAD flag is set, else may be NULL)
 *   iters        : [B]      Newton steps taken (may be NULL)
 *   status       : [B]      enum dcol_status (may be NULL)
 * tol is pdip_tol (reference default 1e-6); max_iter the iteration cap (reference: 50).
 * Asynchronous on `stream` (a hipStream_t, NULL = default stream); no allocation and no
 * synchronisation, so the call can be captured into a hipGraph.                        */
int dcol_plan_run(const dcol_plan* plan, const double* pose1, const double* pose2, double tol,
                  int32_t max_iter, int32_t flags, double* alpha, double* contact, double* grad,
                  int32_t* iters, int32_t* status, void* stream);

/* Convenience: HOST arrays in, HOST arrays out, synchronous.  Array-of-structures rows:
 * pose1/pose2 B x 6, contact B x 3, grad B x 12.  Builds a transient plan; staging
 * buffers are owned by the table (calls on one table are serialised).               */
int dcol_prox_batch_host(const dcol_table* table, int64_t B, const int32_t* shape1,
                         const int32_t* shape2, const double* pose1, const double* pose2,
                         double tol, int32_t max_iter, int32_t flags, double* alpha,
                         double* contact, double* grad, int32_t* iters, int32_t* status);

/* The drop-in's per-call form (proximity/proximity.py:6-54, proximity_gradient.py:91-138:
 * ONE pair per call, which is how the reference's systems call it, per obstacle per knot --
 * systems/cluttered_hallway_quadrotor.py:131-133, :155).  HOST arguments: pose1/pose2 (6),
 * contact (3, if DCOL_CONTACT, else may be NULL), grad (12, if a GRAD flag, else may be NULL),
 * iters / status (may be NULL).  Synchronous.  Latency path: a one-pair plan cached per
 * (shape1, shape2) in the table (its kernel variant), poses and outputs in device-mapped
 * pinned host memory read and written by the GPU itself (no copy commands).  A pair whose
 * variant the fused small-plan kernel has is served by the table's one-pair SERVER: one
 * resident workgroup polling that memory, started by the first such call and leaving after
 * DCOL_PAIR_SERVER_IDLE_US (default 1000) without a request -- no kernel launch per call.
 * (A device-wide synchronisation issued meanwhile waits for it to leave.  The server runs
 * on a CU-masked stream, which HIP gives a hardware queue of its own, so no kernel of
 * another stream queues behind it.)  Other pairs,
 * and every pair under DCOL_PAIR_SERVER=0, take one launch on a stream of the table.
 * Calls on one table are serialised.                                                      */
int dcol_prox_pair(const dcol_table* table, int32_t shape1, int32_t shape2, const double* pose1,
                   const double* pose2, double tol, int32_t max_iter, int32_t flags, double* alpha,
                   double* contact, double* grad, int32_t* iters, int32_t* status);
/* One-pair plans dcol_prox_pair holds (least recently used evicted past DCOL_PAIR_PLANS_MAX,
 * so device memory stays bounded however many distinct shape pairs a caller queries).  */
#define DCOL_PAIR_PLANS_MAX 64
int dcol_table_pair_plans(const dcol_table* table, int32_t* n);
/* Counters of dcol_prox_pair on this table: calls answered by the server, calls that
 * launched their own kernel, server starts, over the served calls the device time from the
 * server seeing a request to its answer (microseconds and shader-clock cycles, sums: their
 * ratio is the clock the solves ran at), and the XCD (0-7) the last server started on (-1:
 * none yet).  Any pointer may be NULL.                                                   */
int dcol_table_pair_stats(const dcol_table* table, int64_t* served, int64_t* launched,
                          int64_t* server_starts, double* server_solve_us, double* server_solve_cycles,
                          int32_t* server_xcd);

/* Diagnostic (the stamps build, `make stamps` -> lib_stamps/): the shader-clock stamps of the
 * last request the pair server answered -- [0..5] solve start, frames, assembly, initialise,
 * PDIP loop end, gradient end; [6] request seen, [7] answer released; [8..15] sub-phases of
 * PDIP iteration 2.  DCOL_ERR_ARG in the product build.                                    */
int dcol_debug_pair_stamps(const dcol_table* table, uint64_t out[16]);
/* Stop this table's pair server now, if one is resident (waiting at most 5 s for it to
 * leave); the next dcol_prox_pair starts a new one.  E.g. before a long batch phase, so no
 * wave polls the mailbox meanwhile.                                                      */
int dcol_table_stop_pair_server(const dcol_table* table);
/* *running = 1 while this table's pair server is resident (its stream has not drained).  */
int dcol_table_pair_server_running(const dcol_table* table, int32_t* running);
/* Stop every resident pair server of the process (each table's, waiting at most 5 s for
 * each to leave) and start no new one: later dcol_prox_pair calls take the launch path.
 * Registered as an exit handler at the first server start, so a process that exits without
 * destroying its tables never tears down its HIP context under a polling wave; callers may
 * also run it themselves before their own teardown (the Python binding does, at atexit).
 * DCOL_DEBUG_SHUTDOWN=1 reports the servers it found running on stderr.  Returns
 * DCOL_ERR_HIP if a server did not leave (its table is then kept).                      */
int dcol_shutdown(void);

/* ---- multi-GPU ------------------------------------------------------
 * One process per GPU.  Pairs are independent, so each rank solves its own shard with its
 * own plan; when one consumer needs the whole batch, dcol_prox_batch_multi_gpu packs the
 * shard's results and performs ONE all-gather (RCCL over xGMI, librccl loaded on first
 * use).  Bootstrap: rank 0 calls dcol_comm_unique_id and ships the 128 bytes to the other
 * ranks by the host's own means (the reference's Python: torch.distributed / a file).
 * The collective library is librccl unless the environment names another one in
 * DCOL_RCCL_LIB when the id / the communicator is made (tests: an in-process stand-in that
 * runs several ranks as threads on one GPU, tests/fake_rccl/).                           */
#define DCOL_COMM_ID_BYTES 128
/* packed per-pair record, 14 x 8 B = 112 B: alpha, grad[12] (float64), then status and iters
 * as two int32 (little-endian: status in the low half) in the last 8-byte slot           */
#define DCOL_REC 14
typedef struct dcol_comm dcol_comm;
int dcol_comm_unique_id(uint8_t id[DCOL_COMM_ID_BYTES]);
/* Collective over the nranks processes (ncclCommInitRank); `device` = this rank's GPU.   */
int dcol_comm_create(const uint8_t id[DCOL_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                     dcol_comm** out);
int dcol_comm_destroy(dcol_comm* comm);
/* Solve this rank's shard (plan over its n pairs; pose1/pose2 SoA [6][n] and the
 * alpha[n] / grad[12][n] (or NULL) / iters[n] / status[n] outputs are device arrays, as
 * dcol_plan_run), pack row i of rec_local[cap][DCOL_REC] = [alpha, grad(12) (NaN without a
 * gradient flag), (int32 status, int32 iters)] (rows n..cap-1 = NaN), then all-gather every rank's
 * rec_local into rec_all[nranks * cap][DCOL_REC] (rank r's rows at r * cap).  Requires
 * n <= cap, the same cap on every rank.  Asynchronous on `stream`; no allocation.
 * rec_local == NULL: in place -- the solver kernels write the records straight into this
 * rank's rows of rec_all (rows n..cap-1: all-ones bytes, i.e. NaN doubles and the int pair
 * (-1, -1)) and the all-gather runs in place (sendbuff = rec_all + rank * cap * DCOL_REC):
 * no pack pass and no local copy.  alpha / grad / iters / status are then optional (NULL:
 * records only; given: filled as well).  flags | DCOL_NO_GATHER (in place only): everything
 * but the all-gather.                                                                    */
int dcol_prox_batch_multi_gpu(const dcol_plan* plan, dcol_comm* comm, const double* pose1, const double* pose2,
                              double tol, int32_t max_iter, int32_t flags, int64_t cap, double* alpha,
                              double* grad, int32_t* iters, int32_t* status, double* rec_local,
                              double* rec_all, void* stream);
/* The in-place all-gather alone: every rank's rows [rank * cap, (rank + 1) * cap) of
 * rec_all[nranks * cap][DCOL_REC] to every rank, asynchronous on `stream` (after a
 * DCOL_NO_GATHER solve; the caller orders the two streams, e.g. with an event).  Issue the
 * collectives of one communicator in the same order on every rank.                      */
int dcol_comm_all_gather(dcol_comm* comm, int64_t cap, double* rec_all, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DCOL_H */
