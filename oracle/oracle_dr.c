/*
 * oracle_dr.c — CPU restatement of the domain-randomization path (test infrastructure only; see
 * oracle.h).  Follows tasks/base/vec_task.py:612-842 (apply_randomizations, the noise lambdas of
 * 684-720) and utils/dr_utils.py:68-170 (generate_random_samples, get_bucketed_val,
 * apply_random_samples), in the layout of include/migym.h (env_props rows, mg_dr_desc / mg_dr_attr).
 * PARITY: the property values and the noise lambdas are pinned to the reference run on the fake gym
 * (tests/golden/trace_ant_dr.npz, make_traces.py) with the reference's numpy / torch draws injected.
 */
#include <math.h>
#include <stdint.h>

#include "oracle.h"

static double sched_scaling(const mg_dr_desc* d, int64_t last_step) { /* dr_utils.py:76-81 */
  if (d->schedule == MG_DR_SCHED_LINEAR)
    return 1.0 / (double)d->schedule_steps * (double)(last_step < d->schedule_steps ? last_step : d->schedule_steps);
  if (d->schedule == MG_DR_SCHED_CONSTANT) return last_step < d->schedule_steps ? 0.0 : 1.0;
  return 1.0;
}

static double draw(const mg_dr_desc* d, double sc, float u1, float u2) { /* dr_utils.py:83-127 */
  double a = d->range[0], b = d->range[1];
  if (d->distribution == MG_DR_GAUSSIAN) {
    if (d->operation == MG_DR_ADDITIVE) { a *= sc; b *= sc; }
    else { b = b * sc; a = a * sc + 1.0 * (1.0 - sc); }
    return a + b * (sqrt(-2.0 * log(1.0 - (double)u1)) * cos(6.283185307179586 * (double)u2));
  }
  if (d->operation == MG_DR_ADDITIVE) { a *= sc; b *= sc; }
  else { a = a * sc + 1.0 * (1.0 - sc); b = b * sc + 1.0 * (1.0 - sc); }
  if (d->distribution == MG_DR_LOGUNIFORM) return exp(log(a) + (log(b) - log(a)) * (double)u1);
  return a + (b - a) * (double)u1;
}

static double bucketed(const mg_dr_desc* d, double v) { /* dr_utils.py:130-139 */
  double lo, hi;
  if (d->distribution == MG_DR_UNIFORM) { lo = d->range[0]; hi = d->range[1]; }
  else { lo = d->range[0] - 2.0 * sqrt((double)d->range[1]); hi = d->range[0] + 2.0 * sqrt((double)d->range[1]); }
  const int nb = d->num_buckets;
  int cnt = 0;
  for (int i = 0; i < nb; i++)
    if ((hi - lo) * (double)i / (double)nb + lo <= v) cnt = i + 1;
  const int idx = cnt - 1 < 0 ? nb - 1 : cnt - 1; /* buckets[bisect(...) - 1], Python index -1 wraps */
  return (hi - lo) * (double)idx / (double)nb + lo;
}

int orc_dr_apply(const mg_dr_apply_args* a) {
  for (int e = 0; e < a->n; e++) {
    int doit = a->first != 0;
    if (!doit) { /* vec_task.py:633-637: randomize_buf >= frequency on a resetting step */
      int64_t rb = a->randomize_buf[e] + (a->increment ? 1 : 0);
      doit = rb >= (int64_t)a->frequency && a->reset_mask[e] != 0;
      if (doit) rb = 0;
      a->randomize_buf[e] = rb;
    }
    if (!doit) continue;
    const uint64_t gid = (uint64_t)(a->env_offset + e);
    float* row = a->env_props + (size_t)a->stride * e;
    for (int i = 0; i < a->nattr; i++) {
      const mg_dr_attr* at = &a->attrs[i];
      const mg_dr_desc* d = &a->descs[at->desc];
      if (!a->first && !d->after_setup) continue; /* setup_only (vec_task.py:800-812) */
      double smp;
      if (a->samples) {
        smp = (double)a->samples[(size_t)a->nattr * e + i];
      } else {
        const float u1 = orc_uniform(a->seed, gid, a->counter, (uint32_t)(8192 + 2 * i));
        const float u2 = orc_uniform(a->seed, gid, a->counter, (uint32_t)(8193 + 2 * i));
        smp = draw(d, sched_scaling(d, a->last_step), u1, u2);
      }
      double v = d->operation == MG_DR_SCALING ? (double)at->og * smp : (double)at->og + smp; /* dr_utils.py:159-162 */
      if (d->num_buckets > 0) v = bucketed(d, v);
      row[at->slot] = (float)v;
    }
  }
  return 0;
}

int orc_dr_noise(const mg_dr_noise_args* a) { /* vec_task.py:684-692 / 711-718, fp32 op order */
  for (int64_t i = 0; i < a->n; i++) {
    const uint64_t gid = (uint64_t)(a->elem_offset + i);
    float c;
    if (a->refresh_corr) {
      if (a->injected_corr) {
        c = a->injected_corr[i];
      } else {
        const float u1 = orc_uniform(a->seed, gid, a->counter, 4 * a->key), u2 = orc_uniform(a->seed, gid, a->counter, 4 * a->key + 1);
        c = sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.28318530717958647f * u2);
      }
      a->corr[i] = c;
    } else {
      c = a->corr[i];
    }
    float z;
    if (a->injected) {
      z = a->injected[i];
    } else {
      const float u1 = orc_uniform(a->seed, gid, a->counter, 4 * a->key + 2);
      if (a->distribution == MG_DR_GAUSSIAN) {
        const float u2 = orc_uniform(a->seed, gid, a->counter, 4 * a->key + 3);
        z = sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.28318530717958647f * u2);
      } else {
        z = u1;
      }
    }
    const float cc = c * a->c_scale + a->c_shift;
    const float nz = (cc + z * a->scale) + a->shift;
    const float x = a->operation == MG_DR_SCALING ? a->x[i] * nz : a->x[i] + nz;
    a->x[i] = x;
    if (a->x_clamped) a->x_clamped[i] = fminf(fmaxf(x, -a->clip), a->clip);
  }
  return 0;
}
