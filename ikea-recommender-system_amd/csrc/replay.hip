// Replay-buffer transitions built on the device from a session store
// (SURVEY §8f rank 2).  The reference materialises every transition's state
// and next state as Python lists in a pandas pickle (replay_buffer.py:24-74,
// built by preprocessing.py:385-489) and collates them per batch on the host;
// here the sessions stay in HBM once, as CSR (items int32 and rewards f64 per
// event, the event's session, session offsets), and a batch of event indices
// becomes the trainers' 7-tuple directly:
//   state      the last min(n_bef, L) items before the event (pad id elsewhere;
//              end padding: items first, begin padding: items last)
//   action     the event's item          reward   the event's reward
//   next_state the last min(n_bef + 1, L) items up to and including it
//   true_len   clamp(n_bef, 1, L)       true_next_len   min(n_bef + 1, L)
//   is_end     the event is its session's last
// with n_bef = the number of earlier events of the session — the rules of
// preprocessing.py:5-29 (get_state), :143-170 (get_next_state), :426-464.
#include "common.h"

__global__ __launch_bounds__(256) void k_build_transitions(
    const int32_t* __restrict__ items, const double* __restrict__ rew, const int32_t* __restrict__ ev_sess,
    const int64_t* __restrict__ sess_off, const int64_t* __restrict__ ev, int B, int L, int64_t pad_id, int pad_end,
    int64_t* __restrict__ s, int64_t* __restrict__ a, double* __restrict__ r, int64_t* __restrict__ s_next,
    int64_t* __restrict__ len, int64_t* __restrict__ next_len, uint8_t* __restrict__ is_end) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per transition
  if (b >= B) return;
  const int64_t e = ev[b];
  const int sess = ev_sess[e];
  const int64_t st = sess_off[sess], en = sess_off[sess + 1];
  const int64_t n_bef = e - st;
  const int64_t take = n_bef < L ? n_bef : L;            // items in the state
  const int64_t take2 = n_bef + 1 < L ? n_bef + 1 : L;   // items in the next state
  const int64_t first = st + n_bef - take, first2 = st + n_bef + 1 - take2;
  for (int j = lane; j < L; j += 64) {
    // position j holds history item (j - shift) with shift = 0 (end padding) or L - take (begin)
    const int64_t jj = pad_end ? j : j - (L - take);
    const int64_t jj2 = pad_end ? j : j - (L - take2);
    s[(int64_t)b * L + j] = (jj >= 0 && jj < take) ? items[first + jj] : pad_id;
    s_next[(int64_t)b * L + j] = (jj2 >= 0 && jj2 < take2) ? items[first2 + jj2] : pad_id;
  }
  if (lane == 0) {
    a[b] = items[e];
    r[b] = rew[e];
    len[b] = n_bef < 1 ? 1 : take;
    next_len[b] = take2;
    is_end[b] = e == en - 1;
  }
}

extern "C" int rg_build_transitions(const int32_t* items, const double* rew, const int32_t* ev_sess,
                                    const int64_t* sess_off, const int64_t* ev, int B, int L, int64_t pad_id,
                                    int pad_end, int64_t* s, int64_t* a, double* r, int64_t* s_next, int64_t* len,
                                    int64_t* next_len, uint8_t* is_end, hipStream_t stream) {
  if (B <= 0 || L <= 0 || !items || !rew || !ev_sess || !sess_off || !ev || !s || !a || !r || !s_next || !len ||
      !next_len || !is_end)
    return RG_ERR_ARG;
  hipLaunchKernelGGL(k_build_transitions, dim3((B + 3) / 4), dim3(256), 0, stream, items, rew, ev_sess, sess_off, ev,
                     B, L, pad_id, pad_end, s, a, r, s_next, len, next_len, is_end);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
