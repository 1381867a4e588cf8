/*
 * swarm.h -- C-ABI of libswarm.so, the MI355X (gfx950) swarm-step library.
 *
 * The reference has no FFI: its boundary is the Python module `agent` whose handlers are
 * called once per message (agent.py:197-214 dispatch).  These entry points replace the
 * *batched* form of those handlers -- one call runs a whole synchronous round (or all rounds
 * to convergence) for every agent at once.  Python binds them with ctypes
 * (distributed-swarm-algorithm_amd/swarm_amd/_lib.py; INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (HBM), borrowed: the library never frees them.
 *     Positions are interleaved float64 pairs (x0, y0, x1, y1, ...), i.e. agent.py:47
 *     `self.position` / task['pos'].
 *   - Agents are addressed by storage index i in [0, n); ids[i] (int32, >= 0, distinct) is
 *     the protocol ID (agent.py:26 `agent_id`).  The storage order is the caller's choice; the
 *     batched Python layer stores agents in spatial (grid-cell) order for locality.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Work is
 *     stream-ordered; the documented host sync points are the host-pointer outputs
 *     (rounds_exec, changes_per_round, stats, n_edges).
 *   - Return 0 (SWARM_OK) on success, > 0 for a soft condition, < 0 on error;
 *     swarm_last_error() returns the calling thread's last message.
 *   - Scratch memory is owned by a swarm_ctx (grows on demand, freed by swarm_ctx_destroy).
 *     A ctx is bound to the device that was current when it was created; one ctx per thread.
 */
#ifndef SWARM_H
#define SWARM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWARM_OK 0
#define SWARM_NOT_CONVERGED 1  /* max_rounds reached without a zero-change round */
#define SWARM_ERR_ARG (-1)     /* invalid argument (sizes, NULL pointers, ranges) */
#define SWARM_ERR_HIP (-2)     /* HIP runtime error (message has the hipError string) */
#define SWARM_ERR_OOM (-3)     /* scratch allocation failed */
#define SWARM_ERR_RANGE (-4)   /* a size exceeds the index type (e.g. >= 2^31 edges) */
#define SWARM_ERR_STALE (-5)   /* swarm_allocate_indexed: positions moved since swarm_cell_index */

/* Agent states as stored in the uint8 state array (agent.py:19-22 AgentState values). */
#define SWARM_FOLLOWER 1
#define SWARM_ELECTION_WAIT 2
#define SWARM_LEADER 3

/* Election execution strategies.  Both are exact: identical leaders, states, rounds_exec
 * and per-round change counts. */
#define SWARM_ELECT_DENSE 0    /* every agent gathers every round (Jacobi sweep) */
#define SWARM_ELECT_FRONTIER 1 /* dense sweeps while many agents change, then only the agents
                                  marked by last round's risers gather (sparse rounds) */
#define SWARM_ELECT_TIMED 0x100 /* OR into mode: time every kernel with HIP events (stats) */
#define SWARM_ELECT_TRUST_C16 0x200 /* OR into mode (swarm_elect_compact*): the caller vouches that col16 was
                                       written by swarm_graph_compact on this ctx from the same row_ptr / col
                                       and n, and that none of the three changed since; the 16-bit column
                                       check and the edge-count read-back are then skipped (no host wait
                                       before the first round).  Without such a record on the ctx the call
                                       checks the columns as usual. */

/* Allocation execution strategies (all exact). */
#define SWARM_ALLOC_AUTO 0
#define SWARM_ALLOC_BINNED 1   /* cell-list candidates within the claim radius */
#define SWARM_ALLOC_DENSE 2    /* every agent x every task, ID-ordered tiles */

typedef struct swarm_ctx swarm_ctx;

/* A uniform cell grid over agent positions (swarm_cell_index). */
typedef struct swarm_grid {
    double xmin, ymin, xmax, ymax;  /* bounding box of the indexed positions */
    double cell, inv_cell;          /* cell side (>= the requested one if the grid was capped) */
    int64_t ncx, ncy;               /* cells per row, rows */
} swarm_grid;

typedef struct swarm_alloc_stats {
    int64_t n_claims;        /* TASK_CLAIM messages the round produced (agent.py:302) */
    int64_t n_conflicts;     /* TASK_CONFLICT messages the resolver emitted (agent.py:322,325) */
    int64_t n_flagged;       /* claims/decisions inside the libm guard band */
    int64_t n_candidates;    /* agent x task pairs evaluated exactly in fp64 */
    int64_t n_overflow;      /* tasks whose claims exceeded the on-chip list (slow exact path) */
    int64_t mode_used;       /* SWARM_ALLOC_BINNED or SWARM_ALLOC_DENSE */
    int64_t n_resolved;      /* tasks with a guard-band pair, decided with the host's libm pow */
} swarm_alloc_stats;

typedef struct swarm_elect_stats {
    int64_t rounds_launched; /* rounds issued (>= rounds_exec; extra ones are no-ops) */
    int64_t active_total;    /* agents gathered (DENSE: all; SPARSE: marked), rounds 1..rounds_exec */
    int64_t edges_total;     /* CSR edges visited, summed over rounds 1..rounds_exec */
    int64_t changes_total;   /* leader changes, summed over rounds */
    double gather_ms;        /* SWARM_ELECT_TIMED: device time of every launched round kernel */
    double apply_ms;         /* always 0 (one kernel per round); kept for layout stability */
    int64_t gather_launches; /* launches behind gather_ms (all launched rounds) */
    int64_t dense_rounds;    /* rounds executed as a full DENSE sweep */
    double bytes_total;      /* algorithmic HBM bytes of rounds 1..rounds_exec */
    double sparse_ms;        /* SWARM_ELECT_TIMED: device time of every launched sparse round */
    int64_t sparse_launches; /* SWARM_ELECT_TIMED: sparse rounds launched (incl. no-ops) */
    double sparse_bytes;     /* algorithmic HBM bytes of the executed sparse rounds */
} swarm_elect_stats;

const char *swarm_last_error(void);
/* "swarm-mi355x <version> (gfx950) src=<16 hex>": the hex digits are the sha256 prefix of the
 * sources the library was built from (csrc/Makefile HASHED), so a stale build is detectable. */
const char *swarm_version(void);

int swarm_ctx_create(swarm_ctx **out);
int swarm_ctx_destroy(swarm_ctx *ctx);

/*
 * Leader election to convergence (contract E2).
 * Replaces: SwarmAgent._handle_election_acclaim (agent.py:263-275) and
 * SwarmAgent._handle_heartbeat (agent.py:243-261) applied by every agent to every
 * neighbour's re-advertised leader each round, starting from the state
 * _check_election_timeout leaves after a win (agent.py:234-241: LEADER, leader_id = id).
 *   round t:  leader[v] <- max(leader[v], max_{u in N(v)} leader[u])   (synchronous)
 *   stop after the first round with zero changes; rounds_exec counts that round.
 *   state[v] = SWARM_LEADER iff leader[v] == ids[v], else SWARM_FOLLOWER.
 * row_ptr/col: CSR of N(v) (who v hears) over storage indices; FRONTIER mode requires it
 * symmetric (a riser marks the agents in its own row) -- use swarm_elect_directed otherwise.
 * leader (device, n): output.  changes_per_round (host, capacity max_rounds, may
 * be NULL): per-round change counts for rounds 1..rounds_exec.  stats (host) may be NULL.
 * Returns SWARM_NOT_CONVERGED if max_rounds rounds all changed something.
 */
int swarm_elect(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col,
                const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds,
                int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                swarm_elect_stats *stats, void *stream);

/* Same for a directed neighbour graph (agent.py:59-65: update_sensors' per-agent neighbour
 * lists need not be symmetric).  hear_row_ptr/hear_col (device) is the transpose of
 * row_ptr/col -- for each agent, the agents that hear it -- through which FRONTIER rounds mark
 * the agents a riser can change next round.  hear_row_ptr[n] must equal row_ptr[n]
 * (SWARM_ERR_ARG otherwise).  DENSE mode ignores it. */
int swarm_elect_directed(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col,
                         const int32_t *hear_row_ptr, const int32_t *hear_col, const int32_t *ids,
                         int32_t *leader, uint8_t *state, int32_t max_rounds, int32_t mode,
                         int32_t *rounds_exec, int64_t *changes_per_round, swarm_elect_stats *stats,
                         void *stream);

/* Compact (16-bit) columns of a symmetric int32 CSR for the elections (an MI355X layout, no reference
 * counterpart): col16[k] = col[k] - (v & ~63) for every edge k of row v, i.e. each neighbour as a
 * delta from its row's 64-agent base.  In a spatial storage order (swarm_cell_order) a neighbour lies
 * within about one grid row of its agent, so the deltas fit and every column read moves half the
 * bytes.  col16 (device, row_ptr[n] int16, caller-allocated).  Returns SWARM_ERR_RANGE (col16
 * unusable) when a delta does not fit in 16 bits.  Rebuild it whenever the graph changes. */
int swarm_graph_compact(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col, int16_t *col16,
                        void *stream);

/* swarm_graph_compact that never refuses: a delta outside [-32767, 32767] is stored as -32768 (an escape)
 * and the elections read that neighbour from the int32 columns (col must stay alive beside col16).  For
 * shard graphs, whose ghost rows sit in blocks away from the owned rows: the frontier stepper
 * takes these columns through swarm_frontier_set_compact_escaped / swarm_shard.col16_escaped.
 * *n_escaped (host): the escaped edges.  < 2^30 edges. */
int swarm_graph_compact_escaped(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col,
                                int16_t *col16, int64_t *n_escaped, void *stream);

/* swarm_elect reading the graph's compact columns (swarm_graph_compact of the same row_ptr/col -- never
 * swarm_graph_compact_escaped's, which only the frontier stepper reads; col16 NULL: same as swarm_elect).  Same results, same stats.  With col16 it takes graphs of up to
 * 2^31 - 2^20 edges (the 16-bit columns' 32-bit byte offsets), so a 1.6e9-edge swarm (C5's 100M agents
 * on one GPU) runs on 32-bit row offsets; without, < 2^30 edges as swarm_elect. */
int swarm_elect_compact(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col, const int16_t *col16,
                        const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds, int32_t mode,
                        int32_t *rounds_exec, int64_t *changes_per_round, swarm_elect_stats *stats, void *stream);

/* Same with int64 row offsets: graphs with >= 2^30 edges or agents (the int32-CSR entry points
 * address with 32-bit byte offsets and reject them with SWARM_ERR_ARG; swarm_elect_compact with
 * 16-bit columns reaches 2^31 - 2^20 edges). */
int swarm_elect_i64(swarm_ctx *ctx, int64_t n, const int64_t *row_ptr, const int32_t *col,
                    const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds,
                    int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                    swarm_elect_stats *stats, void *stream);

/* swarm_elect_compact with int64 row offsets (graphs of >= 2^30 edges; the 16-bit columns are
 * built by swarm_graph_compact from the int32 row offsets, which hold up to 2^31 - 1 edges).
 * Replaces the same election as swarm_elect_i64 (agent.py:263-275); col16 = NULL is swarm_elect_i64. */
int swarm_elect_compact_i64(swarm_ctx *ctx, int64_t n, const int64_t *row_ptr, const int32_t *col,
                            const int16_t *col16, const int32_t *ids, int32_t *leader, uint8_t *state,
                            int32_t max_rounds, int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                            swarm_elect_stats *stats, void *stream);

/* One synchronous E2 round, dense, no convergence loop (building block for sharded runs):
 * leader_out[v] = max(leader_in[v], max_{u in N(v)} leader_in[u]) for v in [0, n_rows);
 * leader_in may hold n_rows + ghosts entries (col indexes it).  *changed (device int64) is
 * incremented by the number of rows whose value rose. */
int swarm_elect_round(swarm_ctx *ctx, int64_t n_rows, const int32_t *row_ptr,
                      const int32_t *col, const int32_t *leader_in, int32_t *leader_out,
                      int64_t *changed, void *stream);

/*
 * Frontier stepper for sharded (multi-GPU) elections: the same exact rounds as
 * swarm_elect(FRONTIER) but driven one round at a time, so a caller can exchange halo values
 * between rounds (swarm_amd/dist.py does it over RCCL).  Local storage = n_rows owned agents
 * followed by ghosts (copies of other shards' boundary agents), n_all in total; the CSR has
 * n_all rows (ghost rows list their local neighbours) and col indexes [0, n_all).
 * Leaders are double-buffered by round parity: round t reads leader[(t-1)&1] and writes
 * leader[t&1], so after round t the current state is leader[t&1] (leader0 / leader1, both
 * n_all, owned by the caller).
 *   begin:   leader0 = leader1 = init; round 1 is a full dense sweep.
 *   step:    round t over the owned rows (dense or sparse, decided on the device from round
 *            t-1's changes + ghost rises; no convergence guard: a shard with no local change
 *            can still receive ghost changes).  Owned changes are counted per round.
 *   ghosts:  after the halo exchange of round t, incoming[i] is the round-t leader of ghost
 *            begin+i; rises are written to both buffers and their local neighbours marked for
 *            round t+1.
 *   changes: per-round owned change counts of rounds t0..t1 (t1 - t0 < 256); host sync.
 *            Read at least every 256 rounds (counter slots are recycled).
 * One stepper per ctx; swarm_elect() on the same ctx resets it.
 */
int swarm_frontier_begin(swarm_ctx *ctx, int64_t n_rows, int64_t n_all, const int32_t *init,
                         int32_t *leader0, int32_t *leader1, void *stream);
/* swarm_frontier_begin with the owned rows at [own_begin, own_begin + n_own) (ghost rows on both
 * sides); swarm_frontier_set_compact: the shard graph's 16-bit columns for the following steps
 * (swarm_graph_compact; NULL: the int32 columns), reset by every begin. */
int swarm_frontier_begin_range(swarm_ctx *ctx, int64_t own_begin, int64_t n_own, int64_t n_all, const int32_t *init,
                               int32_t *leader0, int32_t *leader1, void *stream);
int swarm_frontier_set_compact(swarm_ctx *ctx, const int16_t *col16);
/* The same for swarm_graph_compact_escaped's columns (escaped neighbours read from the step's col). */
int swarm_frontier_set_compact_escaped(swarm_ctx *ctx, const int16_t *col16);
int swarm_frontier_step(swarm_ctx *ctx, int32_t t, const int32_t *row_ptr, const int32_t *col,
                        int32_t *leader0, int32_t *leader1, void *stream);
int swarm_frontier_ghosts(swarm_ctx *ctx, int32_t t, int64_t begin, int64_t count,
                          const int32_t *incoming, const int32_t *row_ptr, const int32_t *col,
                          int32_t *leader0, int32_t *leader1, void *stream);
int swarm_frontier_changes(swarm_ctx *ctx, int32_t t0, int32_t t1, int64_t *out, void *stream);

/*
 * Multi-GPU election: the sharded round loop on the device stream.  Each round:
 * the frontier round over every shard row; after every halo_depth-th round the owned rows each
 * peer keeps as ghosts are packed and sent to it, and the ghosts are received from it (RCCL
 * ncclSend/ncclRecv to EVERY peer in one group), and the received ghost leaders applied
 * (swarm_frontier_ghosts semantics); every batch of rounds one ncclAllReduce(sum) of the
 * per-round owned change counts decides convergence.  Same results as swarm_elect(FRONTIER) on
 * the union graph, for any partition of the agents over the ranks (strips: 2 peers; ID ranges of
 * Morton IDs: a compact region with up to 8; random IDs: every rank).  RCCL is taken from the
 * process at run time (the instance torch loaded); swarm_comm_available() says whether it was found.
 * Replaces: the reference's transport stub (agent.py:188-194) -- it has no multi-process path.
 */
typedef struct swarm_comm swarm_comm;

/* One rank's shard.  Rows: [ghosts of the peers below this rank | owned | ghosts of the peers above]:
 * the ghosts received from peers[j] are the ghost_count[j] rows that follow those of peers[j-1], the
 * peers ranked below this rank filling [0, own_begin) and the peers above [own_begin + n_rows, n_all)
 * (checked).  The ghosts must contain every agent within halo_depth hops of an owned agent, with
 * every edge among the shard's rows in the CSR (swarm_amd/dist.py: every agent within
 * halo_depth radio radii of the owner's region).  A peer appears once even if the halo is empty in
 * one direction; a peer with nothing either way may be left out. */
typedef struct swarm_shard {
    int64_t n_rows;               /* owned agents: rows [own_begin, own_begin + n_rows) */
    int64_t n_all;                /* owned + ghost agents */
    const int32_t *row_ptr;       /* CSR over all n_all rows (ghost rows list their local neighbours) */
    const int32_t *col;
    const int32_t *init;          /* initial leaders = IDs of all n_all agents */
    int64_t own_begin;            /* first owned row */
    int32_t halo_depth;           /* k >= 1 (0 = 1): all n_all rows are stepped, the halo is exchanged
                                     after every k-th round only (owned rows stay exact: a wrong value
                                     starts at the halo's outer edge and moves one hop per round) */
    int32_t n_peers;              /* ranks this shard exchanges with (0 = none) */
    const int32_t *peers;         /* host [n_peers]: their ranks, ascending, none equal to this rank */
    const int64_t *send_count;    /* host [n_peers]: owned rows sent to each peer */
    const int64_t *send_rows;     /* device [sum send_count]: those shard rows, peer after peer */
    const int64_t *ghost_count;   /* host [n_peers]: ghost rows received from each peer */
    const int16_t *col16;         /* swarm_graph_compact of row_ptr / col, or NULL (int32 columns) */
    int32_t col16_escaped;        /* col16 is swarm_graph_compact_escaped's (escapes read from col) */
} swarm_shard;

int swarm_comm_available(void);
int swarm_comm_unique_id(void *out128);
int swarm_comm_create(swarm_comm **out, int nranks, int rank, const void *id128);
int swarm_comm_destroy(swarm_comm *comm);
/* Transport kinds.  SWARM_COMM_RCCL: the calls above (one rank per GPU, RCCL over xGMI).
 * SWARM_COMM_SHM: processes of ONE host, any GPUs (several may share one): the same sharded C loops
 * (swarm_elect_sharded, swarm_auction_sharded) with every exchange staged through a POSIX shared-memory
 * segment and a process-shared barrier (synchronous per op; SWARM_SHM_MB mailbox MiB per rank and
 * parity, default 16; SWARM_SHM_TIMEOUT_S, default 120, before a barrier gives up).  Rank 0 makes the
 * id (swarm_comm_unique_id_kind), every rank passes the same 128 bytes to swarm_comm_create_kind. */
#define SWARM_COMM_RCCL 0
#define SWARM_COMM_SHM 1
int swarm_comm_unique_id_kind(int kind, void *out128);
int swarm_comm_create_kind(swarm_comm **out, int kind, int nranks, int rank, const void *id128);
int swarm_comm_kind(const swarm_comm *comm);
/* leader0 / leader1: n_all each; after rounds_exec rounds the state is leader[rounds_exec&1].
 * changes_per_round (host, capacity max_rounds): GLOBAL per-round change counts. */
int swarm_elect_sharded(swarm_ctx *ctx, swarm_comm *comm, const swarm_shard *shard,
                        int32_t *leader0, int32_t *leader1, int32_t max_rounds,
                        int32_t *rounds_exec, int64_t *changes_per_round, void *stream);
/* swarm_elect_sharded with this rank's own per-round figures (each optional, host, capacity max_rounds):
 * local_counts[3 (r-1) + {0,1,2}] = round r's owned changes, rows gathered and edges gathered on this rank
 * (a dense round: n_all rows and -1 = every edge of the shard graph); round_ms[r-1] = the device time from
 * the start of round r to the start of round r+1 on this rank (one HIP event per round; the per-round cost
 * model of DESIGN §6 is fitted from them).
 * comm may be NULL for a shard without peers (one rank: the shard graph stepped alone). */
int swarm_elect_sharded_ex(swarm_ctx *ctx, swarm_comm *comm, const swarm_shard *shard,
                           int32_t *leader0, int32_t *leader1, int32_t max_rounds,
                           int32_t *rounds_exec, int64_t *changes_per_round, int64_t *local_counts,
                           float *round_ms, void *stream);

/*
 * Task allocation round (contract A-H).
 * Replaces: SwarmAgent._process_tasks + _calculate_utility (agent.py:292-302, 338-347) run by
 * every agent over every OPEN task, then SwarmAgent._handle_task_claim (agent.py:304-325) at
 * the resolver for every claim in ascending sender-ID order, then the winner notification
 * _handle_task_conflict (agent.py:327-336).
 *   U(a,k) = (u_scale / (1 + sqrt(dx*dx + dy*dy))) * has_cap   (fp64, no FMA contraction)
 *   claim iff U > claim_thr; claim value x = f32(U) (round to nearest even)
 *   per task, claims in ascending agent ID: the first claim wins if the task has no current
 *   winner, otherwise a claim replaces the winner iff x > util + hysteresis (fp64).
 *   Guard band: the reference squares with libm pow(|d|, 2.0), which can
 *   differ from d*d by an ulp.  Every task with a pair whose decision or f32 value such an ulp
 *   could change (stats->n_flagged pairs) is deferred; those pairs are decided on the HOST with
 *   this process's libm pow, exactly as agent.py:297/302/340 compute them, and the task is then
 *   resolved once with them (stats->n_resolved tasks; one extra host round trip when > 0).  The
 *   outputs are therefore the reference's on this host's libm, not only the x*x arithmetic's.
 * apos (n*2 f64), acaps (n u32: bit k = capability k), tpos (t*2 f64), treq (t i8: -1 none).
 * winner/util (device, t): in = current claim table (-1 = no claim; util fp64), out = final.
 * won (device, n, may be NULL): out, tasks won per agent.  id_to_index (device, may be NULL,
 * length id_span): storage index of each ID, used to credit `won` for a pre-existing winner
 * that keeps its task.  nclaim/nmsg (device, t, may be NULL): claims and TASK_CONFLICT
 * messages per task.  stats (host, may be NULL).
 */
int swarm_allocate(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos,
                   const uint32_t *acaps, int64_t t, const double *tpos, const int8_t *treq,
                   double claim_thr, double hysteresis, double u_scale, int32_t mode,
                   int32_t *winner, double *util, int32_t *won, const int32_t *id_to_index,
                   int64_t id_span, int64_t *nclaim, int64_t *nmsg, swarm_alloc_stats *stats,
                   void *stream);

/*
 * The same round (BINNED) over agents stored in cell order -- swarm_cell_order's layout, the
 * spatial layout of swarm_amd.Swarm -- without a binning pass: a task's claim window is the
 * grid rows it covers, each a contiguous range of storage indices.  The index comes from
 * swarm_cell_index over the same positions.  Every call verifies on the device that each agent
 * still lies in its cell's range; if not (positions moved since the index was built) it returns
 * SWARM_ERR_STALE and the outputs are undefined -- rebuild the index, or call swarm_allocate.
 * Claim radius (u_scale / claim_thr - 1) must span at most 16 grid rows (SWARM_ERR_ARG).
 */


/* grid (host) and cell_off (device, ncells + 1): agents of cell c = cy * ncx + cx are storage
 * indices [cell_off[c], cell_off[c + 1]).  cell_off == NULL: fill grid and *ncells only.
 * SWARM_ERR_ARG if pos is not in cell order.  Synchronises the stream. */
int swarm_cell_index(swarm_ctx *ctx, int64_t n, const double *pos, double cell, swarm_grid *grid,
                     uint32_t *cell_off, int64_t cell_off_capacity, int64_t *ncells, void *stream);

int swarm_allocate_indexed(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos,
                           const uint32_t *acaps, const swarm_grid *grid, const uint32_t *cell_off,
                           int64_t t, const double *tpos, const int8_t *treq, double claim_thr,
                           double hysteresis, double u_scale, int32_t *winner, double *util,
                           int32_t *won, const int32_t *id_to_index, int64_t id_span,
                           int64_t *nclaim, int64_t *nmsg, swarm_alloc_stats *stats, void *stream);

/* swarm_allocate_indexed with flags (same results):
 *   SWARM_ALLOC_TRUST_INDEX   the caller vouches that apos are the positions swarm_cell_index indexed
 *                             (unchanged since): no device staleness check (never SWARM_ERR_STALE)
 *   SWARM_ALLOC_FRESH_CLAIMS  no claim table: winner / util are outputs only, initialised on the
 *                             device to -1 / 0.0 (what an empty agent.py task_claims table means) */
#define SWARM_ALLOC_TRUST_INDEX 1
#define SWARM_ALLOC_FRESH_CLAIMS 2
int swarm_allocate_indexed_ex(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos,
                              const uint32_t *acaps, const swarm_grid *grid, const uint32_t *cell_off,
                              int64_t t, const double *tpos, const int8_t *treq, double claim_thr,
                              double hysteresis, double u_scale, int32_t flags, int32_t *winner, double *util,
                              int32_t *won, const int32_t *id_to_index, int64_t id_span,
                              int64_t *nclaim, int64_t *nmsg, swarm_alloc_stats *stats, void *stream);

/*
 * Exact fp64 utility for m (agent, task) pairs (agent.py:338-347), GPU arithmetic.
 * out (device, m f64).  Used by parity tests and by callers that need costs, not claims.
 */
int swarm_utility(swarm_ctx *ctx, int64_t m, const double *apos, const uint32_t *acaps,
                  const double *tpos, const int8_t *treq, double u_scale, double *out,
                  void *stream);

/*
 * Radius graph builder (synthetic/sensor input side of the round):
 * edge i~j (i != j) iff dx*dx + dy*dy <= radius*radius (fp64).  Rows ascending.
 * Call with col == NULL to get row_ptr (device, n+1) and *n_edges (host); then again with col
 * (device, capacity col_capacity) to fill.  SWARM_ERR_RANGE (before any row is built) when the
 * cell occupancies say the build would scan more than 2^36 candidate pairs in all or more than
 * 2^20 in one agent's 3 x 3 cell window (co-located agents), or the graph has >= 2^31 edges.
 */
int swarm_build_rgg(swarm_ctx *ctx, int64_t n, const double *pos, double radius,
                    int32_t *row_ptr, int32_t *col, int64_t col_capacity, int64_t *n_edges,
                    void *stream);

/*
 * Spatial storage order: perm (device, n) such that agents perm[0], perm[1], ... are
 * grouped by row-major grid cell of side `cell` (stable within a cell).
 */
int swarm_cell_order(swarm_ctx *ctx, int64_t n, const double *pos, double cell,
                     int32_t *perm, void *stream);

/*
 * Auction allocation (BASELINE config C4) -- the north star's "auction
 * price update": no reference counterpart (the reference allocates by greedy claims and leader
 * hysteresis, swarm_allocate above), parity against the build's CPU restatement
 * (oracle/swarm_oracle.c orc_auction).  One task per agent and one agent per task over the
 * admissible pairs U > claim_thr (agent.py:297), value x = f32(U) (the claim payload,
 * agent.py:302).  Jacobi Bertsekas auction: each round every unassigned, active agent bids on
 * its best task (net = x - price[k], ties -> lowest task index) the price price + (best -
 * second) + eps, where the opt-out option (net 0) competes as a second best; an agent whose
 * best net is <= 0 drops out for good.  Each task takes its highest bid, ties -> lowest agent
 * ID; its previous owner becomes unassigned.  rounds_exec = rounds that had bidders (the auction
 * stops at the first round without one).
 * owner (device, t): storage index of the task's agent or -1; price (device, t, f32);
 * assigned (device, n): task index or -1.  bidders_per_round (host, capacity max_rounds, may be
 * NULL).  Returns SWARM_NOT_CONVERGED if max_rounds rounds all had bidders.
 */
typedef struct swarm_auction_stats {
    int64_t n_pairs;         /* admissible (agent, task) pairs */
    int64_t n_flagged;       /* pairs inside the libm guard band (see swarm_allocate) */
    int64_t rounds_launched; /* rounds issued (>= rounds_exec + 1) */
    int64_t tail_rounds;     /* rounds run by the single-workgroup tail kernel */
    int64_t bids_total;      /* agent-rounds with a bidder, summed over rounds */
} swarm_auction_stats;

int swarm_auction(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos, const uint32_t *acaps,
                  int64_t t, const double *tpos, const int8_t *treq, double claim_thr, double u_scale, float eps,
                  int32_t max_rounds, int32_t *owner, float *price, int32_t *assigned, int32_t *rounds_exec,
                  int64_t *bidders_per_round, swarm_auction_stats *stats, void *stream);

/*
 * Sharded auction (BASELINE config C4 on several GPUs): agents partitioned over
 * ranks, tasks replicated on every rank.  Round r: this rank's unassigned, active agents bid
 * into keys (t task keys, packed as in swarm_auction, + one bidder-count word per rank: t + world
 * u64, zero on the first call), the keys are MAX-all-reduced over ranks, and every rank resolves
 * every task identically.  owner_id holds the owning agent's ID (-1 none; replicated), price is
 * replicated, assigned (n, this rank's agents) the task index or -1.  Results equal
 * swarm_auction over the union of all ranks' agents (rounds, bidder counts, prices, owners).
 *   swarm_auction_begin    candidate lists of this rank's agents; initialises owner_id, price,
 *                          assigned; keeps its state in ctx until the next begin (no other
 *                          libswarm call on this ctx in between)
 *   swarm_auction_bid      round r's bids -> keys (then the caller all-reduces keys with MAX)
 *   swarm_auction_resolve  round r's resolution from the reduced keys; log[r] = the round's global
 *                          bidder count (device int64, indexed by round); zeroes keys again
 *   swarm_auction_sharded  the whole loop on the device stream with an RCCL all-reduce per round
 *                          (comm from swarm_comm_create); returns as swarm_auction
 */
int swarm_auction_begin(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos, const uint32_t *acaps,
                        int64_t t, const double *tpos, const int8_t *treq, double claim_thr, double u_scale, float eps,
                        int32_t *owner_id, float *price, int32_t *assigned, swarm_auction_stats *stats,
                        void *stream);
int swarm_auction_bid(swarm_ctx *ctx, int64_t r, int32_t rank, int32_t world, uint64_t *keys, const float *price,
                      int32_t *assigned, void *stream);
int swarm_auction_resolve(swarm_ctx *ctx, int64_t r, int32_t world, uint64_t *keys, int32_t *owner_id, float *price,
                          int32_t *assigned, int64_t *log, void *stream);
int swarm_auction_sharded(swarm_ctx *ctx, swarm_comm *comm, int64_t n, const int32_t *ids, const double *apos,
                          const uint32_t *acaps, int64_t t, const double *tpos, const int8_t *treq, double claim_thr,
                          double u_scale, float eps, int32_t max_rounds, int32_t *owner_id, float *price,
                          int32_t *assigned, int32_t *rounds_exec, int64_t *bidders_per_round,
                          swarm_auction_stats *stats, void *stream);

/*
 * Physics / formation step: SwarmAgent._update_physics (agent.py:94-181)
 * for every agent, as one synchronous step (contract P1): all agents read the step-start
 * positions pos_in (n x 2 f64) and write pos_out (must differ).  A FOLLOWER (state) with
 * leader_index >= 0 (storage index of its leader, -1 none) targets its V-formation slot behind
 * the f32-rounded leader position (the '!ff' heartbeat payload); target (n x 2 f64) /
 * has_target (n u8) are in/out (agent.py:53 self.target, None = 0).  obstacles: m x 3 f64
 * (x, y, radius), shared by every agent, applied in order; row_ptr/col: each agent's sensed
 * neighbours, applied in CSR order.  vel (n x 2 f64): out for every moving agent.  Agents
 * without a target keep position and velocity (agent.py:113-114).  Arithmetic: fp64, the
 * reference's order of operations, squares as x*x (the reference uses libm pow; <= 1 ulp per
 * square).  n_singular (host, may be NULL): zero distances to an obstacle centre or a
 * neighbour (the reference raises ZeroDivisionError there).
 */
int swarm_physics_step(swarm_ctx *ctx, int64_t n, const int32_t *ids, const uint8_t *state,
                       const int32_t *leader_index, const double *pos_in, double *pos_out, double *vel,
                       double *target, uint8_t *has_target, int64_t m, const double *obstacles,
                       const int32_t *row_ptr, const int32_t *col, double dt, double max_speed,
                       int64_t *n_singular, void *stream);

/*
 * Batched wire codec: the reference's transport framing, agent.py:184-214,
 * for m messages at once.  Big-endian '!BBI' header (type, sender, tick) + payload by type:
 * 1 HEARTBEAT '!ff' (a, b = leader x, y), 2 ELECTION_ACCLAIM '!B' (the sender ID), 3 COORDINATOR
 * (none), 4 TASK_CLAIM '!If' (task, a = utility), 5 TASK_CONFLICT '!IB' (task, winner).
 * wide != 0 widens every u8 ID field to u32 ('!BII' header, '!I' acclaim, '!II' conflict), an
 * extension for swarms with IDs > 255 that the reference cannot frame.
 *
 * encode (device arrays of m; integer fields int64 so out-of-range values are representable):
 * status[i] = 0 ok, 1 struct.error (an integer field out of range), 2 OverflowError (a finite
 * value beyond f32), 3 unknown type -- payload checked before header, as the reference packs
 * them; an errored message takes no bytes.  offsets (device, m+1) = packet offsets into out,
 * offsets[m] = *total_bytes (host).  out == NULL: sizing call (status/offsets/total only);
 * otherwise cap must be >= the total (SWARM_ERR_RANGE: nothing past cap is written).  Synchronises
 * the stream (total_bytes).  One pass: tiles of 2 048 messages take their byte offsets from the lower
 * tiles' published counts (a ticket counter and look-back words in the ctx), so encode calls on one
 * ctx must not overlap (SWARM_ERR_HIP if they did and a look-back gave up).
 */
int swarm_codec_encode(swarm_ctx *ctx, int64_t m, const int64_t *type, const int64_t *sender, const int64_t *tick,
                       const double *a, const double *b, const int64_t *task, const int64_t *winner, int32_t wide,
                       uint8_t *out, int64_t cap, int64_t *offsets, int8_t *status, int64_t *total_bytes,
                       void *stream);

/*
 * decode: packet i is buf[offsets[i] .. offsets[i+1]) (device).  status: 0 handled, 1 dropped
 * (shorter than the header, agent.py:198-199), 2 unknown type (ignored, no handler), 3 the
 * handler's unpack raises struct.error (TASK_CLAIM payload != 8 bytes, TASK_CONFLICT != 5 (8
 * wide)), 4 offsets outside [0, buf_len] or decreasing (packet not read).  Fields not carried by
 * the type are 0; a HEARTBEAT carries a position (has_pos = 1,
 * a/b as f32) only when its payload is exactly 8 bytes (agent.py:256-258).  TASK_CLAIM
 * utility -> a.  Asynchronous on stream.
 */
int swarm_codec_decode(swarm_ctx *ctx, int64_t m, const uint8_t *buf, int64_t buf_len, const int64_t *offsets,
                       int32_t wide,
                       int8_t *status, int64_t *type, int64_t *sender, int64_t *tick, float *a, float *b,
                       int64_t *task, int64_t *winner, uint8_t *has_pos, void *stream);

/*
 * Timer FSM / protocol ticks: every agent's update_loop tick
 * (agent.py:66-80) at once -- inbound ELECTION_ACCLAIM / COORDINATOR / HEARTBEAT handling
 * (243-281) from the CSR neighbours' previous-tick sends, then _check_election_timeout
 * (217-241) and the leader's _send_heartbeat (283-289) -- for ticks t0+1 .. t0+ticks under
 * contract T1 (tools/gen_golden.py ref_fsm): clock = t * dt; agent i's own tick counter is
 * t + tick_off[i] (heartbeats when it is a multiple of 10); the election jitter is
 * jitter * u(seed, id, t) with u the splitmix64 hash of tools/gen_golden.py jitter_u.
 * fsm: device state, in/out (n each unless noted): state (SWARM_*), leader (ID, -1 = None),
 * last_hb / wait_start / delay (f64 seconds: last_heartbeat_time, election_wait_start,
 * election_delay), leader_pos (n x 2 f32, the '!ff' heartbeat payload; (0, 0) when None),
 * has_leader_pos, alive, outbox (2n bytes, tick-parity double buffer: the bytes at parity
 * (t0 & 1) are the tick-t0 sends; bit 0 ACCLAIM+COORDINATOR, bit 1 HEARTBEAT).
 * row_ptr/col: whom each agent hears (its receive order); hear_row_ptr/hear_col: the transpose
 * (who hears each agent; the same arrays for a symmetric graph), or NULL: with it only agents
 * something was sent to walk their row each tick (push marks), without it every agent does.
 * kill_ticks (host, n_kill): at the start of each such tick every alive LEADER dies.
 * counts (host, ticks x 4, may be NULL): per tick, alive LEADERs, alive ELECTION_WAITs, ACCLAIM
 * senders, HEARTBEAT senders.  Synchronises the stream when counts != NULL.
 */
typedef struct {
    uint8_t *state;
    int32_t *leader;
    double *last_hb;
    double *wait_start;
    double *delay;
    float *leader_pos;
    uint8_t *has_leader_pos;
    uint8_t *alive;
    uint8_t *outbox;
} swarm_fsm;

int swarm_protocol_run(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *pos, const int32_t *row_ptr,
                       const int32_t *col, const int32_t *hear_row_ptr, const int32_t *hear_col,
                       const int32_t *tick_off, const swarm_fsm *fsm, int64_t t0, int32_t ticks,
                       double dt, double timeout, double jitter, uint64_t seed, const int64_t *kill_ticks,
                       int32_t n_kill, int64_t *counts, void *stream);

/* swarm_protocol_run with storm ticks pulled and the traffic counted (same results):
 * pull_frac (push mode): when the senders of a tick's workgroup (its share of the agents: a grid-stride
 *   set of 4-agent groups, or of 4 096-agent chunks) exceed pull_frac x its agents, the next tick's
 *   receivers walk their own rows instead of being mailed (a timeout wave makes most agents send at
 *   once: mailing every hearer costs more than every agent pulling); < 0: never.
 * traffic (host, 8 int64, may be NULL; synchronises): summed over the run -- [0] receivers served by
 *   their single sender, [1] receivers that walked their row (several senders), [2] row edges walked
 *   (those and pulled ticks), [3] senders mailed, [4] hearer edges mailed, [5] 0, [6] agents that
 *   walked their row in pulled ticks, [7] pulled ticks.  Pull mode (hear_row_ptr NULL) counts nothing. */
int swarm_protocol_run_ex(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *pos, const int32_t *row_ptr,
                          const int32_t *col, const int32_t *hear_row_ptr, const int32_t *hear_col,
                          const int32_t *tick_off, const swarm_fsm *fsm, int64_t t0, int32_t ticks,
                          double dt, double timeout, double jitter, uint64_t seed, const int64_t *kill_ticks,
                          int32_t n_kill, double pull_frac, int64_t *counts, int64_t *traffic, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* SWARM_H */
