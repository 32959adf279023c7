/* reacher.h -- C ABI of the MI355X-native batched Reacher-v2 environment (libreacher.so).
 *
 * Replaces, for N environments in lockstep on one GPU, the gym env object the reference
 * drivers hold:
 *   make_mujoco_env("Reacher-v2", 0)      reference mlp_train.py:21, lstm_train.py:21
 *   ob = env.reset()                      reference mlp_train.py:112,138,200; lstm_train.py:111,136,196
 *   ob, r, done, _ = env.step(a)          reference mlp_train.py:135,196; lstm_train.py:133,192
 * (gym 0.10.5 ReacherEnv + TimeLimit(50) + baselines Monitor; MuJoCo 1.50 via mujoco-py;
 *  third-party, pinned at reference src/distilation/requirement.txt:5,20,33).
 *
 * Conventions
 *   - Plain pointers and sizes; all array pointers are DEVICE pointers on the handle's
 *     device unless noted.  Calls are asynchronous on the handle's stream (no host sync),
 *     and may be captured in a hipGraph.  One handle per stream; not thread-safe per handle.
 *   - Return 0 on success, RD_EINVAL for a bad argument, -(hipError_t) for a HIP error;
 *     rd_last_error() gives a thread-local message.
 *   - Layouts: obs [N][11] f32 (gym order: cos q0, cos q1, sin q0, sin q1, tx, ty, v0, v1,
 *     fingertip-target x, y, 0), act [N][2] f32, rew [N] f32, done [N] u8,
 *     state [8][N] f32 SoA rows (q0, q1, v0, v1, tx, ty, dx, dy) where (dx, dy) is the
 *     fingertip-target offset at the kinematics MuJoCo holds (the last RK4 stage).
 *   - Lockstep TimeLimit: all envs share the step counter.  The step that reaches 50
 *     returns done=1, the final step's reward, and the RESET observation in obs
 *     (the reference discards the terminal observation and resets: mlp_train.py:137-138).
 */
#ifndef REACHER_H
#define REACHER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RD_OK 0
#define RD_EINVAL (-100000)
#define RD_ECOMM (-100001)   /* a gradient exchange failed (reacher_comm.h); the step's update was skipped */

/* reset draw sources */
#define RD_RESET_PHILOX 0   /* Philox4x32-10(seed, env_base + i, episode): synthetic targets */
#define RD_RESET_TABLE 1    /* host-provided draws (gym MT19937 seeding, see rd_gym_reset_draws) */

typedef struct rd_env rd_env;

/* Create N envs on `device`, asynchronous on `hip_stream` (hipStream_t; NULL = default).
 * env_base: global id of env 0 (ranks shard contiguous ranges).  No reset is done. */
int rd_create(rd_env** out, int64_t n_envs, int64_t env_base, uint64_t seed, int device,
              void* hip_stream);
int rd_destroy(rd_env* env);
/* Subsequent launches go to `hip_stream` (e.g. a graph-capture stream). */
int rd_set_stream(rd_env* env, void* hip_stream);

/* env.reset() for all N envs (episode counter += 1 after the first reset). */
int rd_reset(rd_env* env, float* obs);

/* env.step(a) for all N envs. */
int rd_step(rd_env* env, const float* act, float* obs, float* rew, uint8_t* done);

/* Parity / checkpoint hooks.  step = steps taken in the current episode (0..49). */
int rd_set_state(rd_env* env, const float* state, int32_t step, int32_t episode);
int rd_get_state(rd_env* env, float* state, int32_t* step, int32_t* episode);

/* Reset source.  RD_RESET_TABLE: draws [n_episodes][N][6] f32 device buffer
 * (q0, q1, v0, v1, tx, ty) owned by the caller, kept alive while in use. */
int rd_set_reset_mode(rd_env* env, int mode, const float* draws, int32_t n_episodes);

/* HOST function: gym seeding for one env (gym/utils/seeding.py hash_seed -> MT19937
 * init_by_array) followed by n_episodes ReacherEnv.reset_model draws, in f64.
 * out: host buffer [n_episodes][6] (q0, q1, v0, v1, tx, ty). */
int rd_gym_reset_draws(uint64_t seed, int32_t n_episodes, double* out);

/* HOST function: CRC32C (Castagnoli, reflected 0x82F63B78) of n bytes of host memory,
 * continuing from `crc` (0 to start) -- the checksum of the TF1 V2 checkpoint bundles the
 * reference's tf.train.Saver writes (lstm_train.py:86-107,199; teacher.py:17-20), computed
 * natively for tf_checkpoint.py (slicing-by-8). */
uint32_t rd_crc32c(const uint8_t* data, int64_t n, uint32_t crc);

/* Which kernel variant / library build is loaded (for provenance checks). */
const char* rd_version(void);
const char* rd_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
