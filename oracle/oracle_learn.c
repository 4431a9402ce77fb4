/* oracle_learn.c -- CPU restatement of DQNAgent.learn (TEST INFRASTRUCTURE).
 *
 * src/agents/dqn_agent.py:328-380 with the Keras 3.9 / TF 2.19 semantics it
 * relies on (un-vendored: keras 3.9.2 uv.lock:283-284, tensorflow 2.19.0
 * uv.lock:999-1000; restated from their published algorithms):
 *   q-network  dqn_agent.py:153-184  Dense(H1,relu) Dense(H2,relu) Dense(4)
 *              y = x W + b, kernels [fan_in][fan_out] (Keras layout)
 *   :342       a* = argmax online(S')   (first max on ties, tf.argmax)
 *   :343-345   q_t = target(S')[a*]
 *   :347       y = r + gamma * (1 - d) * q_t
 *   :350-352   q = sum(online(S) * one_hot(A)); loss = mean((y - q)^2)
 *              loss_kind 1: Keras Huber (delta 1; the loss of
 *              src/experimental/agent.py:99): e = q - y,
 *              mean(|e| <= 1 ? 0.5 e^2 : |e| - 0.5), dL/dq = clip(e, -1, 1) / B
 *   :356-357   gradients; keras.optimizers.Adam.update_step:
 *              m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
 *              w -= (m * alpha) / (sqrt(v) + eps),
 *              alpha = lr * sqrt(1 - b2^t) / (1 - b1^t)
 * fp32 throughout (the reference computes under mixed_float16; the fp32
 * restatement is the stricter oracle, tolerances are stated in the tests).
 * TF/Keras are absent.  The restatement is pinned by tests/golden/learn.npz:
 * the reference's own DQNAgent.learn control flow run over a torch-backed TF
 * shim (tests/golden/make_learn_golden.py, tf_shim.py), 393 MSE and 233 Huber
 * learns (tests/test_learn_golden_cpu.py); and cross-checked against torch
 * autograd in tests/test_learn_oracle_cpu.py.
 *
 * Parameter vector (Keras get_weights order): W1[89][H1] b1[H1] W2[H1][H2]
 * b2[H2] W3[H2][NA] b3[NA].
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define D_IN 89

long orc_qnet_nparams(int H1, int H2, int NA) {
    return (long)D_IN * H1 + H1 + (long)H1 * H2 + H2 + (long)H2 * NA + NA;
}

/* forward of B rows; optional caches z1,z2 (pre-activation) [B][H] */
void orc_qnet_forward(const float *p, int H1, int H2, int NA, const float *x, int B, float *q,
                      float *z1c, float *z2c) {
    const float *W1 = p, *b1 = W1 + D_IN * H1, *W2 = b1 + H1, *b2 = W2 + H1 * H2;
    const float *W3 = b2 + H2, *b3 = W3 + H2 * NA;
    float *h1 = (float *)malloc(sizeof(float) * H1), *h2 = (float *)malloc(sizeof(float) * H2);
    for (int b = 0; b < B; b++) {
        const float *xb = x + (size_t)b * D_IN;
        for (int j = 0; j < H1; j++) {
            float s = 0.0f;
            for (int i = 0; i < D_IN; i++) s += xb[i] * W1[i * H1 + j];
            s += b1[j];
            if (z1c) z1c[(size_t)b * H1 + j] = s;
            h1[j] = s > 0.0f ? s : 0.0f;
        }
        for (int k = 0; k < H2; k++) {
            float s = 0.0f;
            for (int j = 0; j < H1; j++) s += h1[j] * W2[j * H2 + k];
            s += b2[k];
            if (z2c) z2c[(size_t)b * H2 + k] = s;
            h2[k] = s > 0.0f ? s : 0.0f;
        }
        for (int a = 0; a < NA; a++) {
            float s = 0.0f;
            for (int k = 0; k < H2; k++) s += h2[k] * W3[k * NA + a];
            q[(size_t)b * NA + a] = s + b3[a];
        }
    }
    free(h1);
    free(h2);
}

static int argmax_first(const float *q, int n) {
    int best = 0;
    for (int a = 1; a < n; a++)
        if (q[a] > q[best]) best = a;
    return best;
}

/* One learn step.  Returns the loss; updates p, m, v in place.
 * hyper: [gamma, alpha_t, c1=(1-b1), c2=(1-b2), eps]; grad_out (optional) [P] */
float orc_learn(float *p, const float *target, float *m, float *v, int H1, int H2, int NA,
                int B, const float *S, const int32_t *A, const float *Rn, const float *S2,
                const float *Dn, const float *hyper, float *grad_out, int loss_kind) {
    const float gamma = hyper[0], alpha = hyper[1], c1 = hyper[2], c2 = hyper[3], eps = hyper[4];
    long P = orc_qnet_nparams(H1, H2, NA);
    float *q2 = (float *)malloc(sizeof(float) * B * NA), *qt = (float *)malloc(sizeof(float) * B * NA);
    float *q = (float *)malloc(sizeof(float) * B * NA), *y = (float *)malloc(sizeof(float) * B);
    float *z1 = (float *)malloc(sizeof(float) * B * H1), *z2 = (float *)malloc(sizeof(float) * B * H2);
    float *g = (float *)calloc(P, sizeof(float));
    orc_qnet_forward(p, H1, H2, NA, S2, B, q2, NULL, NULL);
    orc_qnet_forward(target, H1, H2, NA, S2, B, qt, NULL, NULL);
    for (int b = 0; b < B; b++) {
        int as = argmax_first(q2 + b * NA, NA);
        float tq = qt[b * NA + as];
        float gd = gamma * (1.0f - Dn[b]);
        y[b] = Rn[b] + gd * tq;
    }
    orc_qnet_forward(p, H1, H2, NA, S, B, q, z1, z2);
    const float *W2 = p + D_IN * H1 + H1, *W3 = W2 + H1 * H2 + H2;
    float *gW1 = g, *gb1 = gW1 + D_IN * H1, *gW2 = gb1 + H1, *gb2 = gW2 + H1 * H2;
    float *gW3 = gb2 + H2, *gb3 = gW3 + H2 * NA;
    float loss = 0.0f;
    float *dz2 = (float *)malloc(sizeof(float) * H2), *dz1 = (float *)malloc(sizeof(float) * H1);
    for (int b = 0; b < B; b++) {
        float pred = q[b * NA + A[b]];
        float diff = pred - y[b];
        float dq;
        if (loss_kind == 1) {
            float ae = fabsf(diff);
            loss += ae <= 1.0f ? 0.5f * diff * diff : ae - 0.5f;
            dq = (ae <= 1.0f ? diff : (diff > 0.0f ? 1.0f : -1.0f)) / (float)B;
        } else {
            loss += diff * diff;
            dq = 2.0f * diff / (float)B;
        }
        const float *z1b = z1 + (size_t)b * H1, *z2b = z2 + (size_t)b * H2;
        for (int k = 0; k < H2; k++) {
            float h2 = z2b[k] > 0.0f ? z2b[k] : 0.0f;
            gW3[k * NA + A[b]] += h2 * dq;
            dz2[k] = z2b[k] > 0.0f ? dq * W3[k * NA + A[b]] : 0.0f;
            gb2[k] += dz2[k];
        }
        gb3[A[b]] += dq;
        for (int j = 0; j < H1; j++) {
            float h1 = z1b[j] > 0.0f ? z1b[j] : 0.0f;
            float s = 0.0f;
            for (int k = 0; k < H2; k++) {
                gW2[j * H2 + k] += h1 * dz2[k];
                s += dz2[k] * W2[j * H2 + k];
            }
            dz1[j] = z1b[j] > 0.0f ? s : 0.0f;
            gb1[j] += dz1[j];
        }
        const float *xb = S + (size_t)b * D_IN;
        for (int i = 0; i < D_IN; i++)
            for (int j = 0; j < H1; j++) gW1[i * H1 + j] += xb[i] * dz1[j];
    }
    loss /= (float)B;
    for (long i = 0; i < P; i++) {
        float gi = g[i];
        m[i] = m[i] + (gi - m[i]) * c1;
        v[i] = v[i] + (gi * gi - v[i]) * c2;
        p[i] = p[i] - (m[i] * alpha) / (sqrtf(v[i]) + eps);
    }
    if (grad_out) memcpy(grad_out, g, sizeof(float) * P);
    free(q2); free(qt); free(q); free(y); free(z1); free(z2); free(g); free(dz2); free(dz1);
    return loss;
}
