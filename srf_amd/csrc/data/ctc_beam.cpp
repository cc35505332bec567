// CTC prefix beam search for the SRF decode step (include/srf_data.h), host C++.
//
// Replaces tf.nn.ctc_beam_search_decoder as process_test_step calls it
// (trainer_sr.py:109-112: time-major logits, sequence_length = inp_len // 4,
// beam_width = --decoding-beam-width, top_paths = 1).  TF's decoder
// (tensorflow/core/util/ctc/ctc_beam_search.h, un-vendored, TF >= 2.3) takes raw
// logits, normalises each frame with a log-softmax, treats class C-1 as the blank,
// and keeps per-prefix log probabilities split into "ends in blank" and "ends in a
// label"; the v2 op does not merge repeats of the decoded path again.  Per frame:
//   blank:     P_b(l)    += P(l) * y_blank
//   repeat:    P_nb(l)   += P_nb(l) * y_last(l)
//   extend c:  P_nb(l+c) += (c == last(l) ? P_b(l) : P(l)) * y_c
// over the beams kept at the previous frame, then the beam_width prefixes with the
// largest P = P_b + P_nb are kept (ties: the earlier-created prefix).  Prefixes are
// nodes of a trie, so a beam is an int and extension is a hash lookup.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <unordered_map>
#include <vector>

#include "../../../include/srf_data.h"

namespace {

constexpr float kNegInf = -std::numeric_limits<float>::infinity();

inline float log_sum_exp(float a, float b) {
  if (a == kNegInf) return b;
  if (b == kNegInf) return a;
  const float m = std::max(a, b);
  return m + std::log1p(std::exp(-std::fabs(a - b)));
}

struct Node {
  int parent;
  int label;   // -1 at the root
};

struct Score {
  float pb, pnb;
  float total() const { return log_sum_exp(pb, pnb); }
};

}  // namespace

extern "C" int srf_ctc_beam_search(const float* logits, int T, int C, int blank, int beam_width, int32_t* out_labels,
                                   int* out_len, float* out_log_prob) {
  if (T < 0 || C < 2 || blank < 0 || blank >= C || beam_width < 1 || !out_len || (T > 0 && (!logits || !out_labels)))
    return -1;
  std::vector<Node> nodes{{-1, -1}};
  std::unordered_map<uint64_t, int> child;   // (parent, label) -> node
  auto child_of = [&](int parent, int c) {
    const uint64_t key = (uint64_t)(uint32_t)parent << 32 | (uint32_t)c;
    auto it = child.find(key);
    if (it != child.end()) return it->second;
    const int id = (int)nodes.size();
    nodes.push_back({parent, c});
    child.emplace(key, id);
    return id;
  };
  std::vector<int> beams{0};
  std::vector<Score> score{{0.f, kNegInf}};   // indexed by beam slot
  std::vector<float> lp(C);
  std::unordered_map<int, int> slot;          // node -> index into next
  std::vector<int> next_nodes;
  std::vector<Score> next_score;
  for (int t = 0; t < T; ++t) {
    const float* x = logits + (size_t)t * C;
    float mx = x[0];
    for (int c = 1; c < C; ++c) mx = std::max(mx, x[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += std::exp(x[c] - mx);
    const float norm = mx + std::log(se);
    for (int c = 0; c < C; ++c) lp[c] = x[c] - norm;
    slot.clear();
    next_nodes.clear();
    next_score.clear();
    auto at = [&](int node) -> Score& {
      auto it = slot.find(node);
      if (it != slot.end()) return next_score[it->second];
      slot.emplace(node, (int)next_nodes.size());
      next_nodes.push_back(node);
      next_score.push_back({kNegInf, kNegInf});
      return next_score.back();
    };
    for (size_t k = 0; k < beams.size(); ++k) {
      const int n = beams[k];
      const Score s = score[k];
      const float tot = s.total();
      const int last = nodes[n].label;
      {
        Score& d = at(n);
        d.pb = log_sum_exp(d.pb, tot + lp[blank]);
        if (last >= 0) d.pnb = log_sum_exp(d.pnb, s.pnb + lp[last]);
      }
      for (int c = 0; c < C; ++c) {
        if (c == blank) continue;
        const float prev = (c == last) ? s.pb : tot;
        if (prev == kNegInf) continue;
        Score& d = at(child_of(n, c));
        d.pnb = log_sum_exp(d.pnb, prev + lp[c]);
      }
    }
    // keep the beam_width most probable prefixes (stable: creation order breaks ties)
    std::vector<int> order(next_nodes.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::vector<float> tot(next_nodes.size());
    for (size_t i = 0; i < tot.size(); ++i) tot[i] = next_score[i].total();
    const size_t keep = std::min(order.size(), (size_t)beam_width);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return tot[a] > tot[b]; });
    beams.resize(keep);
    score.resize(keep);
    for (size_t i = 0; i < keep; ++i) {
      beams[i] = next_nodes[order[i]];
      score[i] = next_score[order[i]];
    }
  }
  size_t best = 0;
  for (size_t i = 1; i < beams.size(); ++i)
    if (score[i].total() > score[best].total()) best = i;
  std::vector<int32_t> rev;
  for (int n = beams[best]; n > 0; n = nodes[n].parent) rev.push_back(nodes[n].label);
  *out_len = (int)rev.size();
  for (size_t i = 0; i < rev.size(); ++i) out_labels[i] = rev[rev.size() - 1 - i];
  if (out_log_prob) *out_log_prob = score[best].total();
  return 0;
}
