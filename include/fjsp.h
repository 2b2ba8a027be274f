/*
 * fjsp.h — C-ABI of the MI355X-native vectorised FJSP environment (libfjsp.so).
 *
 * One handle = N independent reference environments stepped in lockstep by hand-written
 * HIP kernels for gfx950, one wavefront lane per environment, all state resident in HBM
 * as SoA arrays.  Plain pointers and sizes only; no torch types.  All device pointers are
 * owned by the caller (e.g. torch tensors' data_ptr()); the library owns the state buffers.
 * Every call is stream-ordered on the handle's hipStream_t and does not synchronise unless
 * documented.  Return value: 0 = OK, < 0 = API error (message via fjsp_last_error()).
 * Simulation anomalies never fail a call; they are reported per env in `status` bits.
 *
 * Reference interfaces replaced (FARIDKH/Multi-agent-RL-for-FJSP):
 *   fjsp_create      <- FJSPSimulation.__init__            FJSPSimulation.py:41-59
 *                       FJSPParallelEnv.__init__            FJSPParallelEnvWrapper.py:27-33
 *   fjsp_reset       <- FJSPSimulation.reset                FJSPSimulation.py:286-323
 *                       FJSPParallelEnv.reset               FJSPParallelEnvWrapper.py:43-54
 *   fjsp_step        <- FJSPSimulation.step                 FJSPSimulation.py:144-242
 *                       (agents/ execute_action, SimPy run, RewardModel, get_observations)
 *   fjsp_step_many   <- K x FJSPSimulation.step with random actions (train.py:268 sample())
 *   fjsp_gae         <- MultiAgentTransitionMemory.finish_trajectory transition_memory.py:45-105
 *   fjsp_gae_shared  <- the same over the batched A2C's memories (one critic value per env)
 *   fjsp_a2c_policy_step <- MultiAgentA2C.learn's collect step: predict -> env.step -> memory.put
 *                       a2c.py:284-309 (one launch per vector step)
 *   fjsp_pack_a2c    <- MultiAgentA2C._get_global_state / _flatten_obs  a2c.py:118-166
 *   FJSP_ACTIONS_HEURISTIC <- MultiAgentA2C._get_heuristic_actions     a2c.py:390-537
 *   fjsp_read_env    <- FJSPSimulation.get_order_progress   FJSPSimulation.py:260-284
 *                       + agv.position / agv.carrying_tray / current_step (a2c.py:298-376)
 *
 * Python binding (ctypes) lives in multi-agent-rl-for-fjsp_amd/_native.py; see INTEGRATION.md.
 */
#ifndef FJSP_H
#define FJSP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FJSP_ABI_VERSION 12

#define FJSP_NUM_AGENTS 8      /* pickup, agv, small, big, pkg_blue_1, pkg_blue_2, pkg_red, pkg_green */
#define FJSP_OBS_I32 20        /* pickup 7 + agv 13 (position = 2) int32 observation fields */
#define FJSP_OBS_I8 12         /* 6 stations x {is_busy, queue_length} int8 fields */
#define FJSP_OBS_F32 6         /* 6 stations x processing_progress float32 */
#define FJSP_MASKS 29          /* action masks: 3 + 8 + 6 x 3 int8 */
#define FJSP_A2C_FEATS 38      /* a2c global state: per agent sorted keys w/o action_mask (a2c.py:118-166) */
#define FJSP_MAX_ORDERS 64     /* num_orders limit per episode */
#define FJSP_ACTION_ABSENT 255 /* agent missing from the action dict (no execute_action call) */

/* status bits (per env, sticky until reset) */
#define FJSP_STATUS_DIVERGED     0x1u   /* a path the reference would raise on / that is not emulated */
#define FJSP_STATUS_OBS_OVERFLOW 0x2u   /* int8 obs > 127 (numpy OverflowError in the reference) */
#define FJSP_STATUS_PKG_WAIT     0x4u   /* packaging request exceeded Resource capacity (not emulated) */
#define FJSP_STATUS_TRAY_LOST    0x8u   /* storage full: dropped tray lost (reference behaviour) */
#define FJSP_STATUS_PROD_LOST    0x10u  /* no packaging station with capacity: products lost (reference behaviour) */
#define FJSP_STATUS_OVERWRITE    0x20u  /* machine START overwrote an unsignalled tray (reference behaviour) */
#define FJSP_STATUS_SLOT_OVERFLOW 0x40u /* more trays in one episode than the slot arena holds (not emulated) */
#define FJSP_STATUS_SPIN_TIMEOUT 0x80u  /* a wave of a multi-wave step kernel gave up waiting for another wave's
                                           hand-off (bounded wait; results of that workgroup are invalid) */

/* action_mode for fjsp_step_many */
#define FJSP_ACTIONS_UNMASKED 0  /* uniform over the full action space (action_space.sample()) */
#define FJSP_ACTIONS_MASKED   1  /* uniform over the valid actions of the current mask */
#define FJSP_ACTIONS_HEURISTIC 2 /* MultiAgentA2C._get_heuristic_actions (a2c.py:390-537) */

typedef struct fjsp_config {
    int32_t num_trays;          /* CONFIG['num_trays'] 1000; pool = min(num_trays, 1000) (FJSPSimulation.py:96) */
    int32_t tray_capacity;      /* CONFIG['tray_capacity'] 5 used by Tray.is_full (1..7) */
    int32_t mask_tray_capacity; /* global CONFIG['tray_capacity'] read by the pickup mask (PickupStationAgent.py:169) */
    int32_t storage_capacity;   /* config.get('storage_capacity', 100) */
    int32_t step_size;          /* CONFIG['step_size'] 10 */
    int32_t max_episode_steps;  /* config.get('max_episode_steps', 500); CONFIG 200 (<= 253) */
    int32_t agv_speed;          /* CONFIG['agv_speed'] 1; 8 / speed must be < step_size */
    int32_t pt_small;           /* PROCESSING_TIMES 60  (multiple of step_size) */
    int32_t pt_big;             /* PROCESSING_TIMES 120 (multiple of step_size) */
    int32_t pt_packaging;       /* PROCESSING_TIMES 30  (multiple of step_size) */
    int32_t packaging_capacity; /* simpy.Resource(capacity=20) (PackagingAgent.py:46) */
} fjsp_config;

/* RewardModel weights (utils/RewardModel.py:12-32; a dataclass of tunable fp64 fields).
 * Rewards: g = ORDER*orders_done + THROUGHPUT*packaged + TIME*step_size (calculate_global_reward),
 * r_a = g / 8 + local_a (combine_rewards), local sums in calculate_local_reward's order. */
typedef struct fjsp_reward_weights {
    double order_complete_reward;     /* 100.0 */
    double throughput_bonus;          /* 10.0 */
    double time_penalty;              /* -0.1 */
    double pickup_load_reward;        /* 1.0 */
    double pickup_tray_complete;      /* 5.0 */
    double pickup_idle_penalty;       /* -1.0 */
    double agv_delivery_reward;       /* 2.0 */
    double agv_move_penalty;          /* -0.1 */
    double agv_packaging_delivery;    /* 10.0 */
    double agv_invalid_action;        /* -5.0 */
    double machine_complete_reward;   /* 5.0 */
    double machine_start_reward;      /* 1.0 */
    double machine_idle_penalty;      /* -2.0 */
    double packaging_complete_reward; /* 20.0 */
    double packaging_start_reward;    /* 2.0 */
    double packaging_idle_penalty;    /* -1.0 */
} fjsp_reward_weights;

/* Output buffers (device pointers).  Each array is [T][F][N] (field-major SoA, N fastest);
 * T = 1 for fjsp_reset / fjsp_step, K for fjsp_step_many.  Any pointer may be NULL (skip). */
typedef struct fjsp_out {
    int32_t* obs_i32;       /* [T][20][N] */
    int8_t* obs_i8;         /* [T][12][N] */
    float* obs_f32;         /* [T][6][N]  */
    int8_t* masks;          /* [T][29][N] */
    double* rewards;        /* [T][8][N]  fp64, RewardModel.combine_rewards */
    uint8_t* term;          /* [T][N] */
    uint8_t* trunc;         /* [T][N] */
    uint32_t* results;      /* [T][8][N] action-result bits (bit 7 = executed; bits 16.. value) */
    int32_t* orders_completed; /* [T][N] infos['orders_completed'] */
    int32_t* packaged;      /* [T][N] infos['total_products_packaged'] */
    double* sim_time;       /* [T][N] infos['sim_time'] */
    uint32_t* status;       /* [T][N] */
    /* observation after auto-reset (== obs for envs that did not finish); [T][F][N] */
    int32_t* next_i32;
    int8_t* next_i8;
    float* next_f32;
    int8_t* next_masks;
    /* a2c global-state features of the observation after auto-reset (the one the policy acts
     * on next): f32 [T][38][N], columns in _get_global_state order (a2c.py:153-166): agents in
     * possible_agents order, each agent's keys sorted, action_mask dropped (_flatten_obs
     * a2c.py:137-151).  Agent a's actor input = columns [off_a, off_a + dim_a) with
     * off = 0,7,20,23,26,29,32,35. */
    float* feats;
} fjsp_out;

/* Host view of one env (fjsp_read_env). */
typedef struct fjsp_env_view {
    int32_t current_step;
    int32_t num_orders;
    int32_t next_order;          /* orders[next_order:] are still in the pickup order_queue */
    int32_t orders_completed;
    int32_t total_packaged;
    int32_t agv_row, agv_col;
    int32_t agv_carrying;        /* 1 if carrying a tray */
    int32_t agv_tray_count;
    uint32_t status;
    /* per order: n | type<<4 | color<<6 | processed_count<<8 | packaged_count<<12 | complete<<16 */
    uint32_t orders[FJSP_MAX_ORDERS];
} fjsp_env_view;

typedef struct fjsp_handle fjsp_handle;

int fjsp_abi_version(void);
const char* fjsp_last_error(void);
int fjsp_default_config(fjsp_config* cfg);
int fjsp_default_reward_weights(fjsp_reward_weights* w);
/* Replace the handle's reward weights (takes effect at the next launch). */
int fjsp_set_reward_weights(fjsp_handle* h, const fjsp_reward_weights* w);
/* Validate a config (0 = usable by the closed-form kernels). */
int fjsp_check_config(const fjsp_config* cfg);

int fjsp_create(const fjsp_config* cfg, int32_t num_envs, int32_t device, void* hip_stream,
                fjsp_handle** out);
int fjsp_destroy(fjsp_handle* h);
int fjsp_set_stream(fjsp_handle* h, void* hip_stream);
/* Tuning knobs: "fused_lds" (-1/0/1, default -1 = auto, on while N <= 16384: stage the per-env
 * tables of k_step_many in LDS, one 64-env workgroup per CU); "pipeline" (0/1, default 1: lean
 * outputs use the two-wave pipelined kernel); "staged_stores" (0/1, default 0: k_step_many stages each
 * step's obs / masks / rewards / term / trunc / status in LDS and writes them as 16-byte
 * chunks; used when only those outputs are requested, N % 64 == 0 and rows are aligned);
 * "timing" (0/1, default 1: bracket fjsp_step / fjsp_step_many launches with hipEvents for
 * fjsp_last_kernel_ms; set 0 while capturing the calls into a hipGraph); "predraw" (0/1,
 * default 1: the pipelined kernel with LDS tables and auto-reset draws every env's next order
 * table ahead on a fourth wave, so auto-resets need no MT draws on the critical path; the
 * results are identical either way); "agents" (0/1, default 1: uniform-random actions with LDS
 * tables and the pre-draw run k_step_ag, the env's agents split over eight wavefronts of its
 * workgroup; identical results); "ag_envs" (0/16/32/64, default 0 = auto: envs per k_step_ag
 * workgroup, lanes >= ag_envs idle; auto = 64 for launches of fewer than 64 steps, else the
 * fewest that give every workgroup a CU of its own; identical results); "step_envs" (0/16/32/64,
 * default 0 = 64; ABI 12: envs per k_step workgroup (fjsp_step), lanes >= step_envs idle;
 * identical results); "env_id_base" (0..2^32-1, default 0: the handle is the shard [value, value + N) of a
 * larger job — every env's MT19937 stream is re-seeded to np.random.seed(value + e), exactly
 * the stream env value + e of one big handle starts from; stream-ordered); "spin_cap"
 * (256..2^31-1, default 2^22: sleep iterations, checked every 256 a wave of a multi-wave step kernel waits for another
 * wave's hand-off before it gives up and flags FJSP_STATUS_SPIN_TIMEOUT / fjsp_faults); "test_stall"
 * (0..2^20, default 0; tests only: later k_step_ag and k_step_pipe<lds,2emit,predraw> launches
 * run a test build in which workgroup 0's owner wave sleeps value x ~8k cycles before its first
 * step, so that the other waves' bounded waits give up and the give-up path runs).  spin_cap and test_stall are not part of a snapshot.
 * Library-wide (h may be NULL; ABI 10): "policy_xmap" (0..3, default 0), "policy_dedup" (0/1,
 * default 1), "policy_split" (0/1, default 1) — the variants of the A2C policy launches listed at
 * fjsp_a2c_policy; "wgrad_waves" (8/16, default 16; ABI 12) — fjsp_a2c_wgrad's workgroups of 8 or
 * 16 waves; identical results.  Nothing is read from the process environment. */
int fjsp_set_option(fjsp_handle* h, const char* name, int64_t value);
int fjsp_num_envs(const fjsp_handle* h);
/* Bytes of device state per env (HBM footprint of the SoA state). */
int64_t fjsp_state_bytes(const fjsp_handle* h);

/* Reset the envs selected by env_mask (device u8[N], NULL = all).  seeds: device u32[N] ->
 * np.random.seed(seeds[e]) first; NULL = continue each env's MT19937 stream (seed=None).
 * Writes the initial observation of the reset envs to out (T = 1; may be NULL). */
int fjsp_reset(fjsp_handle* h, const uint32_t* seeds, const uint8_t* env_mask, int32_t num_orders,
               const fjsp_out* out);

/* One step of every env.  actions: device u8[8][N] (agent-major), 255 = agent absent,
 * other out-of-range values behave as the reference's invalid actions.  agent_order: host
 * u8[8] execution order (the action dict's key order) or NULL = canonical order.
 * autoreset != 0: envs that terminate/truncate are reset (MT stream continued) after their
 * outputs are written; next_* receive the post-reset observation. */
int fjsp_step(fjsp_handle* h, const uint8_t* actions, const uint8_t* agent_order, int32_t autoreset,
              const fjsp_out* out);

/* Step server (ABI 10; FJSPSimulation.step / FJSPParallelEnv.step called once per Python
 * iteration, a2c.py:294): a persistent kernel keeps the handle's envs resident (state words in
 * registers, reward table in LDS, tables warm in L2) and runs one fjsp_step in the canonical dict
 * order per fjsp_server_step, signalled through a doorbell word in host memory — no launch and no
 * stream synchronisation per step.  fjsp_server_start(h, actions, autoreset, out): actions =
 * u8[8][N] the caller rewrites before every fjsp_server_step (pinned host memory, or device memory
 * whose writes are complete), out = the outputs of every step (pinned host memory or device
 * memory; T = 1); N <= 16384.  fjsp_server_step: one step of every env, returns when every output
 * of it is visible to the host.  Any other call on the handle (reset, fjsp_step, read_env,
 * snapshot, set_reward_weights, ...) first stops the server (its state is written back); the next
 * fjsp_server_step relaunches it with the same actions / outputs, as it does after 2 ms without a
 * request (the kernel itself leaves after 5 ms idle, so a device-wide synchronisation issued
 * between steps waits at most that long).  fjsp_server_stop: leave now.
 * Inline mode (ABI 11; one-env handles, the N = 1 drop-in): fjsp_server_start(h, NULL, ...), then
 * fjsp_server_step_actions(h, actions) with the step's 8 action bytes (any host memory): they ride
 * in the doorbell's cache line, so the kernel's poll that sees the request already holds them (one
 * bus round trip per step fewer).  fjsp_server_step on an inline server, or step_actions on one
 * started with an actions buffer, is an error. */
int fjsp_server_start(fjsp_handle* h, const uint8_t* actions, int32_t autoreset, const fjsp_out* out);
int fjsp_server_step(fjsp_handle* h);
int fjsp_server_step_actions(fjsp_handle* h, const uint8_t* actions);
int fjsp_server_stop(fjsp_handle* h);

/* K fused steps with on-device synthetic actions from the counter RNG
 *   h = fmix64(action_seed ^ fmix64(((uint64)(env_gid0 + e) << 32) | (step0 + k)))
 * (spec: oracle/fjsp_oracle.c oracle_actions).  Outputs are [K][F][N] trajectories. */
int fjsp_step_many(fjsp_handle* h, int32_t K, uint64_t action_seed, uint32_t env_gid0, uint32_t step0,
                   int32_t action_mode, int32_t autoreset, const fjsp_out* traj);

/* Discounted returns + GAE over a rollout buffer (transition_memory.py:83-105), fp64,
 * Python operation order.  Columns m = a*N + e (agent-major like the step outputs):
 *   rewards f64[T][M], values f32[T][M], done u8[T][N] (episode ended at t -> next value 0
 *   and a new trajectory starts at t+1), boot f64[M] = next value after t = T-1 (ignored
 *   where done[T-1]).  ret/adv f64[T][M].  M must be a multiple of N. */
int fjsp_gae(const double* rewards, const float* values, const uint8_t* done, const double* boot,
             int32_t T, int32_t N, int32_t M, double gamma, double lamb, double* ret, double* adv,
             void* hip_stream);

/* MT19937 stream of one env in numpy's convention: key = np.random.get_state()[1] (624
 * words), pos = get_state()[2].  Lets the N=1 facade share numpy's GLOBAL legacy RNG with
 * the caller exactly as the reference does (np.random.seed / randint / choice,
 * FJSPSimulation.py:107-112,298-299).  Synchronous. */
int fjsp_mt_get(fjsp_handle* h, int32_t env, uint32_t* key, int32_t* pos);
int fjsp_mt_set(fjsp_handle* h, int32_t env, const uint32_t* key, int32_t pos);

/* Same scan with fp64 values (transition_memory accepts arbitrary Python floats). */
int fjsp_gae_f64(const double* rewards, const double* values, const uint8_t* done, const double* boot,
                 int32_t T, int32_t N, int32_t M, double gamma, double lamb, double* ret, double* adv,
                 void* hip_stream);
/* The same scan with one value per env shared by its agents (the batched A2C: every agent's memory
 * holds the critic's value of the env's global state, a2c.py:300-310,321-332): values f32
 * [T + 1][N], row T = the bootstrap value after t = T-1; rewards / ret / adv f64 [T][agents * N],
 * columns m = a*N + e.  Bit-identical to fjsp_gae with values[t][a*N + e] = values[t][e] and
 * boot[a*N + e] = (double)values[T][e]. */
int fjsp_gae_shared(const double* rewards, const float* values, const uint8_t* done, int32_t T, int32_t N,
                    int32_t agents, double gamma, double lamb, double* ret, double* adv, void* hip_stream);

/* Synchronous host copy of one env's state summary (debug / facade use). */
int fjsp_read_env(fjsp_handle* h, int32_t env, fjsp_env_view* out);
/* Wait for all work queued on the handle's stream. */
int fjsp_sync(fjsp_handle* h);
/* a2c features (f32 [38][N], see fjsp_out.feats) and action masks (int8 [29][N]) of every env's
 * current observation; either pointer may be NULL.  Stream-ordered. */
int fjsp_pack_a2c(fjsp_handle* h, float* feats, int8_t* masks);
/* Source of each a2c feature column: out[38] = index into [obs_i32(20) | obs_i8(12) | obs_f32(6)]
 * (host-only; lets callers and tests check the layout). */
int fjsp_a2c_layout(int32_t* out);
/* Env-state snapshot (every env's packed state, order table, tray-slot arena and MT19937
 * stream): fjsp_snapshot copies fjsp_snapshot_bytes(h) bytes to `dst` (device or host
 * memory), fjsp_restore loads a snapshot taken from a handle with the same num_envs.  Both
 * are stream-ordered (hipMemcpyAsync; pinned host memory for overlap).  The handle's fault
 * word and options (spin_cap, test_stall) are not restored: they stay the handle's.  The role
 * of FJSPSimulation's Python objects being copied / pickled by a caller. */
int64_t fjsp_snapshot_bytes(const fjsp_handle* h);

/* ---- fused A2C policy step (a2c.py:168-252 predict for all agents and envs; networks.py) ----
 * feats f32 [38][N] (fjsp_out.feats layout), masks int8 [29][N]; weights pre-split and pre-packed
 * (ABI 5): every K >= 16 matrix W [R][K] as three bf16 planes hi = bf16(W), mid = bf16(W - hi),
 * lo = bf16(W - hi - mid) (round to nearest even) in MFMA order P(W) = [R/32][K/16][3][64 lanes][8]
 * bf16, element (t, kb, p, l, j) = plane p of W[32 t + (l & 31)][16 kb + 8 (l >> 5) + j]
 * (3 R K / 2 floats of the buffer); biases and the VALU layers as f32:
 *   actor_w: 8 agents x FJSP_POLICY_ACTOR_FLOATS: P(W1 [256][16], inputs zero-padded) | b1 [256] |
 *            P(W2 [256][256]) | b2 [256] | W3 [8][256] (rows >= n_a zero) | b3 [16]
 *   critic_w: P(W1 [256][48], inputs zero-padded) | b1 [256] | P(W2 [256][256]) | b2 [256] |
 *            P(W3 [128][256]) | b3 [128] | W4 [128] | b4 [16]
 * Out: actions u8 [8][N] (argmax if deterministic, else an inverse-CDF draw from the masked
 * distribution keyed by (*seed, env_gid0 + env, step, agent) — the env's global id, so the
 * shards of a multi-GPU job draw independent streams; `seed` is a DEVICE pointer so a captured
 * hipGraph can be re-keyed between replays), values f32 [N], optional masked
 * probabilities f32 [8][8][N] (NULL to skip).  actions == NULL: the critic's values only (masks,
 * actor_w and seed may then be NULL; e.g. the batch-end bootstrap V(s_T), a2c.py:321-332);
 * values == NULL: the actors only (critic_w may be NULL).  Stream-ordered on `stream`.
 * Variants read per launch (fjsp_set_option(NULL, ...); outputs bit-identical under every setting):
 * policy_xmap 0..3 (workgroup -> XCD order; 1-3 also turn the split below off), policy_dedup 0
 * (the station agents' MLP on every env instead of once per distinct input of a 64-env tile),
 * policy_split 0 (fjsp_a2c_policy_step: the pickup station's and the AGV's tiles on one 64-env
 * workgroup instead of two 32-env ones). */
#define FJSP_POLICY_ACTOR_DPAD 16
#define FJSP_POLICY_CRITIC_DPAD 48
#define FJSP_POLICY_ACTOR_FLOATS (3 * 256 * 16 / 2 + 256 + 3 * 256 * 256 / 2 + 256 + 8 * 256 + 16)
#define FJSP_POLICY_CRITIC_FLOATS (3 * 256 * 48 / 2 + 256 + 3 * 256 * 256 / 2 + 256 + 3 * 128 * 256 / 2 + 128 + 128 + 16)
int fjsp_a2c_policy(const float* feats, const int8_t* masks, int32_t n, const float* actor_w, const float* critic_w,
                    const uint64_t* seed, uint32_t env_gid0, uint32_t step, int32_t deterministic, uint8_t* actions,
                    float* values,
                    float* probs, void* stream);
/* One vector step of the A2C collect in ONE launch (a2c.py:284-309: predict -> env.step ->
 * memory): fjsp_a2c_policy's actions (and, when values != NULL, the critic's values) for the
 * handle's n envs, then FJSPSimulation.step (fjsp_step, canonical agent order) of every 64-env
 * tile with those actions, run inside the same launch by the tile's last actor workgroup.
 * feats / masks = the current observation ([38][n] / [29][n]); actions u8 [8][n] and values f32
 * [n] as fjsp_a2c_policy writes them (probabilities are not available here).  out: the step's
 * outputs of this one step, limited to rewards, term, trunc, status, next_masks and feats (each
 * [F][n], any may be NULL; the other fields must be NULL).  Results equal fjsp_a2c_policy
 * followed by fjsp_step with the same arguments, byte for byte.  Replaces fjsp_a2c_policy +
 * fjsp_step per vector step (one launch instead of two).  Only the envs [env_begin, env_begin +
 * env_count) are processed (whole 64-env tiles: env_begin a multiple of 64, env_count a multiple
 * of 64 or reaching n; pointers stay those of all n envs), so that launches over disjoint env
 * ranges can run concurrently on different streams; stream NULL = the handle's stream. */
int fjsp_a2c_policy_step(fjsp_handle* h, const float* feats, const int8_t* masks, const float* actor_w,
                         const float* critic_w, const uint64_t* seed, uint32_t env_gid0, uint32_t step,
                         int32_t deterministic, uint8_t* actions, float* values, int32_t autoreset,
                         const fjsp_out* out, int32_t env_begin, int32_t env_count, void* hip_stream);
/* The critic's forward over n samples for the A2C update (a2c.py:692-699 critic(global_states)
 * over the batch; a2c_vec._CriticGrouped): x f32 [n][40] (ABI 8: sample-major rows, 38
 * features + 2 ignored words, the layout of fjsp_a2c_group_keys' rows; ABI 7 took [38][n]
 * feature rows), critic_w packed as for fjsp_a2c_policy -> values f32 [n] and the post-ReLU hidden
 * layers the backward reads, h1 / h2 f32 [n][256], h3 f32 [n][128] (sample-major).  Same
 * arithmetic as fjsp_a2c_policy's values.  Stream-ordered. */
int fjsp_a2c_critic_forward(const float* x, int32_t n, const float* critic_w, float* h1, float* h2, float* h3,
                            float* values, void* stream);
/* The shard learner's combiner keys (multi-agent-rl-for-fjsp_amd/shard_learner.py, exchange="shard";
 * a2c.py:647-731 with the learner sharded by network; ABI 9): per (agent a, sample s = t n + e)
 * info [8][S] i32 = the agent's action-mask bits | action << 8 and the record key tk [8][S] =
 * fmix64(key_a ^ fmix64(info * 0x9E3779B97F4A7C15 + 1)) over fjsp_a2c_group_keys' actor keys
 * [9][S]; masks int8 [T][29][n], actions u8 [T][8][n]; bad [ceil(S / 256)] i32 set to 1 (never
 * cleared) where a mask byte is neither 0 nor 1.  Stream-ordered. */
int fjsp_a2c_shard_keys(const uint64_t* keys, const int8_t* masks, const uint8_t* actions, int32_t T, int32_t n,
                        uint64_t* tk, int32_t* info, int32_t* bad, void* stream);
/* The grouped update's batch statistics from the GAE outputs ret / adv f64 [T][8][N] in one pass
 * (ABI 9): rsum / rsq f64 [T][N] = per sample the sums over the 8 agents of the f32-rounded
 * return and of its square (calc_critic_loss's FloatTensor(returns), a2c.py:713-722), part f64
 * [T][ceil(N / 256)][8][2] = per-workgroup sums of the f32-rounded advantage and of its square
 * per agent (calc_actor_loss's normalisation, a2c.py:724-731).  Either input may be NULL (its
 * outputs are then not written).  Stream-ordered. */
int fjsp_a2c_slab_stats(const double* ret, const double* adv, int32_t T, int32_t N, double* rsum, double* rsq,
                        double* part, void* stream);
/* Weights into the policy / critic kernels' operand layout (a2c_vec.pack_mfma; ABI 9): W f32
 * [B][R][K] (transposed = 1: a [B][K][R] source packed as its transpose) -> out [B][R/32][K/16]
 * [3][64][8] bf16 (as floats: [.., 3, 64, 4]), element (b, t, kb, p, l, j) = plane p of the
 * three-bf16 split of W[b][32 t + (l & 31)][16 kb + 8 (l >> 5) + j] (hi = bf16(x), mid =
 * bf16(x - hi), lo = bf16(x - hi - mid), round to nearest even).  R % 32 == 0, K % 16 == 0.
 * Stream-ordered. */
int fjsp_a2c_pack_mfma(const float* W, int32_t B, int32_t R, int32_t K, int32_t transposed, float* out, void* stream);
/* The shard learner's actor loss head over one agent's records (shard_learner.owner_losses; the
 * per-agent actor loss of a2c.py:724-731 with a record standing for n samples of equal (input,
 * mask, action) whose normalised advantages sum to w; ABI 9): pu f32 [8][umax] = the agent's
 * probabilities per distinct input, inv i64 [R] = each record's input group, info i32 [R] = mask
 * bits | action << 8, wsum f64 [R], cnt i32 [R] -> grad f32 [nact][R] = dL / dp_j per record and
 * sums f64 [ceil(R / 256)][2] = per-block partial sums of (w logp, n entropy).  Stream-ordered. */
int fjsp_a2c_record_head(const float* pu, int32_t umax, const int64_t* inv, int32_t R, int32_t nact, const int32_t* info,
                         const double* wsum, const int32_t* cnt, float inv_count, float ent_coef, float* grad,
                         double* sums, void* stream);
/* The grouped update's critic loss and its backward in one pass over n distinct global states
 * (a2c.py:683-699 critic(global_states), 713-722 calc_critic_loss; ABI 9): x f32 [n][40] as for
 * fjsp_a2c_critic_forward, coef f64 [n][3] = (a, b, c) with state u's share of the loss
 * a/2 V^2 + b V + c (a = 2 n_u / count, b = -2 sum R / (8 count), c = sum R^2 / (8 count)), so
 * dL / dV = a V + b; critic_w, w3t, w2t packed as for fjsp_a2c_policy / fjsp_a2c_critic_backward.
 * Writes h1 / h2 f32 [n][256] (post-ReLU), g3 [n][128], g2 / g1 [n][256] (the pre-activation
 * gradients: the split-K weight gradients' operands), per 32-state tile part f32 [tiles][772] =
 * layer 1 | 2 | 3 bias gradients (256 | 256 | 128), w4's gradient (128), b4's gradient, 3 zeros,
 * loss f64 [tiles] (partial sums), values f32 [n] (may be NULL).  x, h1, h2, g3, g2, g1, part
 * 16-byte aligned.  Stream-ordered. */
int fjsp_a2c_critic_fused(const float* x, int32_t n, const float* critic_w, const float* w3t, const float* w2t,
                          const double* coef, float* h1, float* h2, float* g3, float* g2, float* g1, float* part,
                          double* loss, float* values, void* stream);
/* The critic's weight gradients over the batch's distinct states (the backward of
 * networks.CentralizedCriticNetwork's Linear layers, a2c.py:692-699 critic_loss.backward(); ABI 12;
 * replaces three split-K f32 GEMMs): out f32 [m][ldo] columns < nout = g^T x over U rows,
 * g f32 [U][ldg] (m features: 256 or 128, fjsp_a2c_critic_fused's g1 / g2 / g3), x f32 [U][ldx]
 * (nx features, nx % 4 == 0: the 40-word rows of fjsp_a2c_group_keys (layer 1, nx <= 64, m = 256)
 * or h1 / h2 (68 <= nx <= 256)); nout <= nx.  f32-level products (three bf16 planes, six plane
 * products, as fjsp_a2c_policy), split over P workgroups of 32-sample stages whose partials
 * part f32 [P][m][npad] (npad = 256 if nx > 64 else 64) are summed in a fixed order in f64:
 * deterministic.  g, x 16-byte aligned.  Stream-ordered. */
int fjsp_a2c_wgrad(const float* g, int32_t m, int64_t ldg, const float* x, int32_t nx, int64_t ldx, int64_t U,
                   float* part, int32_t P, float* out, int32_t nout, int64_t ldo, void* stream);
/* The critic's backward through its two 256-wide ReLU layers for the A2C update (a2c.py:692-699
 * critic_loss.backward(); a2c_vec._CriticGrouped): g3 f32 [n][128] (layer 3's pre-activation
 * gradient, fjsp_a2c_value_head_grad), h1 / h2 from fjsp_a2c_critic_forward, w3t / w2t = W3^T
 * [256][128] / W2^T [256][256] packed as the forward's weights -> g2 = (g3 W3) * [h2 > 0], g1 =
 * (g2 W2) * [h1 > 0] f32 [n][256] and their column sums per 32-sample tile, bias_part2 /
 * bias_part1 f32 [ceil(n / 32)][256].  Stream-ordered. */
int fjsp_a2c_critic_backward(const float* g3, const float* h1, const float* h2, int32_t n, const float* w3t,
                             const float* w2t, float* g2, float* g1, float* bias_part2, float* bias_part1, void* stream);
/* Grouping keys of the A2C update (a2c.py:647-703 _update over a batch; a2c_vec.A2CLosses
 * dedup): feats f32 [T][38][n] (the rollout's a2c features) -> keys u64 [9][T * n], row a < 8
 * a hash of actor a's padded input (its a2c.py:118-134 observation block, zero-padded to 13
 * columns), row 8 of the critic's 38-column global state (a2c.py:153-166); equal inputs get
 * equal keys (the caller verifies the grouping).  Stream-ordered on `stream`. */
int fjsp_a2c_group_keys(const float* feats, int32_t T, int32_t n, uint64_t* keys, float* rows, void* stream);
/* rows (ABI 8; may be NULL, else 16-byte aligned): f32 [T * n][40], each sample's 38 features as
 * a sample-major row (2 zero words of padding), written by the same pass: the input of
 * fjsp_a2c_group_verify.
 * The check of that grouping: rep_a int64 [8][T * n] / rep_c int64 [T * n] = the representative
 * sample of each sample's actor-input / global-state group, rows = fjsp_a2c_group_keys' rows
 * (ABI 8; ABI 7 read the feature-major slab: 38 scattered words per representative).  bad int32
 * [ceil(T * n / 256)] = 1 for a block of 256 samples holding one whose inputs differ bitwise from
 * its representative's (a hash collision: the caller falls back to the dense update), else 0.
 * Stream-ordered. */
int fjsp_a2c_group_verify(const float* rows, int32_t T, int32_t n, const int64_t* rep_a, const int64_t* rep_c,
                          int32_t* bad, void* stream);
/* The grouping itself (ABI 8; a2c_vec.RowGroups on the GPU): keys uint64 [R][S] (R <= 16,
 * R * S < 2^31, fjsp_a2c_group_keys' rows) -> per row the distinct keys as groups, numbered in
 * sorted key order, the samples sorted by group with equal keys in sample order (stable), each
 * group's first sample and run end.  fjsp_a2c_group_sort: one radix sort of every row's 59 key
 * bits with the row id above them (flat / sorted uint64 [R * S], pos / spos uint32 [R * S]), the
 * run starts (runs uint32 [R * S]) and their inclusive scan (scan), and the group count of each
 * row, counts int64 [R]; temp: fjsp_a2c_group_temp_bytes(R * S) bytes.  lowcard (ABI 10): bit r
 * set = row r is expected to hold at most 64 distinct keys (the station agents' rows) and is
 * grouped by a stable counting sort instead (same outputs); a row that turns out to hold more
 * reports counts[r] = -1 and the caller groups again with that bit clear.  After the caller has read
 * counts and chosen umax >= every count, fjsp_a2c_group_runs: starts (scratch) / first / ends int64
 * [R][umax] (padding groups: start and end S, first = the row's last sorted sample), perm int64
 * [R][S] (sample of each sorted position), inv int64 [R][S] (group of each sample), rep int64
 * [R][S] (first sample of each sample's group).  Stream-ordered. */
int fjsp_a2c_group_temp_bytes(int64_t count, uint64_t* bytes);
int fjsp_a2c_group_sort(const uint64_t* keys, int32_t R, int64_t S, uint32_t lowcard, void* temp, uint64_t temp_bytes,
                        uint64_t* flat, uint64_t* sorted, uint32_t* pos, uint32_t* spos, uint32_t* runs, uint32_t* scan,
                        int64_t* counts, void* stream);
int fjsp_a2c_group_runs(const uint32_t* spos, const uint32_t* scan, int32_t R, int64_t S, int64_t umax, int64_t* starts,
                        int64_t* perm, int64_t* inv, int64_t* rep, int64_t* first, int64_t* ends, int32_t* gsorted,
                        void* stream);
/* (gsorted int32 [R][S]: the group of each sorted position.)  The backward of a per-group gather
 * over that grouping (a2c.py:692-699: the gradient of every sample's network output summed into
 * its distinct input): out f32 [J][umax] = per group g of row rowmap[j], the sum in f64 over its
 * samples in sorted order of vals[j][sample] (* scale[j] in f32 first; scale may be NULL).  temp:
 * fjsp_a2c_run_sums_bytes(J, S) bytes.  Deterministic.  Stream-ordered. */
int fjsp_a2c_run_sums_bytes(int32_t J, int64_t S, uint64_t* bytes);
int fjsp_a2c_run_sums(const float* vals, int32_t J, const int32_t* rowmap, const float* scale, const int64_t* perm,
                      const int32_t* gsorted, int64_t S, int64_t umax, void* temp, uint64_t temp_bytes, float* out,
                      void* stream);
/* The actor loss head of the grouped update (a2c.py:204-220 masked probabilities, :705-731
 * entropy and calc_actor_loss): pu f32 [8][8][umax] = each agent's action probabilities per
 * distinct input, inv int64 [8][T * n] = each sample's distinct input, masks int8 [T][29][n],
 * actions u8 [T][8][n] and adv f64 [T][8][n] (the rollout slab's and GAE's layouts; sample
 * s = t * n + e), adv_mean / adv_std f32 [8] (the advantages are used as
 * (float(adv) - mean) / (std + 1e-8), calc_actor_loss a2c.py:724-731; both NULL: float(adv)
 * as is).  Out: grad f32
 * [29][T * n] = d(sum_a actor_loss_a) / d(sample probabilities), row mask_off[a] + j for agent
 * a's valid action j (the 29 action-mask columns' order), and sums f64
 * [8][ceil(T * n / 256)][2] = per agent and block of 256 samples (sum adv_n * logp, sum
 * entropy); the caller adds the blocks.  Stream-ordered. */
int fjsp_a2c_actor_head(const float* pu, int32_t umax, const int64_t* inv, int32_t T, int32_t n, const int8_t* masks,
                        const uint8_t* actions, const double* adv, const float* adv_mean, const float* adv_std,
                        float inv_count, float ent_coef, float* grad, double* sums, void* stream);
/* ReLU backward fused with the bias gradient (the critic backward of the A2C update,
 * a2c.py:713-722 calc_critic_loss through the 256-256-128 ReLU layers): gy, y f32 [rows][cols]
 * (y = the layer's ReLU output), cols 128 or 256.  Out: g f32 [rows][cols] = gy where y > 0
 * else 0, part f32 [ceil(rows / 128)][cols] = column sums of g per block of 128 rows (the
 * caller adds the blocks).  Stream-ordered. */
int fjsp_a2c_relu_bias_grad(const float* gy, const float* y, int64_t rows, int32_t cols, float* g, float* part,
                            void* stream);
/* Backward of the critic's last two layers (a2c.py:153-166 critic 256 -> 128 ReLU -> 1):
 * y f32 [rows][128] = the 128-wide ReLU output, gv f32 [rows] = d loss / d value, w4 f32 [128]
 * = the value head's weights.  Out: g f32 [rows][128] = gv w4 where y > 0 else 0 (the gradient
 * at the 128-wide layer's pre-activation), part f32 [ceil(rows / 128)][260] per block of 128
 * rows: [0, 128) column sums of g (bias gradient), [128, 256) sums of gv y (w4's gradient),
 * [256] sum of gv (the value bias's gradient), [257, 260) zero.  Stream-ordered. */
int fjsp_a2c_value_head_grad(const float* y, const float* gv, const float* w4, int64_t rows, float* g, float* part,
                             void* stream);
int fjsp_snapshot(fjsp_handle* h, void* dst);
int fjsp_restore(fjsp_handle* h, const void* src);
/* Kernel timing of the last fjsp_step_many / fjsp_step / fjsp_a2c_policy_step launch in ms
 * (hipEvents on the handle's stream; synchronises).  A fjsp_a2c_policy_step launched on another
 * stream is not timed (it leaves the previous value). */
int fjsp_last_kernel_ms(fjsp_handle* h, float* ms);
/* Name of the kernel variant the last fjsp_step / fjsp_step_many launched ("" before any):
 * e.g. "k_step_pipe<lds>" (rocprof shows it as k_step_pipe). */
const char* fjsp_last_kernel(const fjsp_handle* h);
/* Fault word of the handle's multi-wave step kernels (k_step_ag, k_step_pipe with hand-offs;
 * not changed by fjsp_restore):
 * bit 0 = some workgroup's wave gave up a bounded wait for another wave's hand-off (its envs
 * also carry FJSP_STATUS_SPIN_TIMEOUT).  Never set by a correct kernel: the bound (option
 * "spin_cap", sleep iterations, default 2^22 ~ 0.1 s) exists so that a hand-off bug ends the
 * launch with a flag instead of hanging the device.  Synchronises; clear != 0 zeroes the word.
 * (No reference counterpart: the reference's agents run sequentially in one Python thread.) */
int fjsp_faults(fjsp_handle* h, uint32_t* out, int32_t clear);

#ifdef __cplusplus
}
#endif
#endif /* FJSP_H */
