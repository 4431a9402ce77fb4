// qnet_layout.hpp -- per-agent parameter layout of the Q-network in HBM.
//
// The reference's Keras model (src/agents/dqn_agent.py:153-184) keeps
// kernels as [fan_in][fan_out].  On the device every agent's parameters (and
// its target copy and Adam m / v) are stored TRANSPOSED, [fan_out][fan_in],
// exactly the reference's 89*H + H*H + 4*H + 2*H + 4 floats (no padding):
//   W1T[H][0..87] (tiled) | W1T[H][88] | W2T[H][H] (tiled) | W3T[4][H] | b1[H] | b2[H] | b3[4]
// W1T and W2T are TILED (qn_wt): 16 x 16 (fan-out x fan-in) tiles of 1 KB in
// row-major tile order, each stored as [fan-in / 8 (2)][fan-out (16)][fan-in % 8 (8)]:
//   (a) a forward MFMA A-fragment (8 consecutive fan-in values of one neuron)
//       is 32 contiguous bytes;
//   (b) a weight-gradient tile C[in][out] produced by MFMA holds 4 consecutive
//       fan-in values per lane, and the 64 lanes' 16-byte Adam accesses cover
//       the tile's 1 KB contiguously (row-major [fan_out][fan_in] gave 16
//       separate 64-byte pieces per wave-instruction: 17 % slower learn).
// Layer 1's 89 inputs are 5.5 tiles + one column: features 0..87 fill five
// whole tiles and the first half (80..87) of a sixth per 16 neurons (qn_w1,
// 1408 floats per 16 neurons), and feature 88 is a separate [H] column.  The
// kernels treat features 89..95 of their 96-wide fragments as zero weights
// without storing them (an earlier layout padded W1T to [H][96]: 896 dead
// floats per agent, ~3 % of the learn kernel's HBM traffic).
// W3T stays row-major.  Host helpers (dmdqn_amd/agent.py) convert to/from the
// Keras get_weights order.
#pragma once

namespace dmdqn {

constexpr int QN_D = 89;    // observation dim (order_lanes.py:554)
constexpr int QN_DP = 96;   // padded feature stride of an observation row (replay ring, X image)
constexpr int QN_DT = 88;   // layer-1 features held in tiles (11 groups of 8); feature 88 is a column
constexpr int QN_NA = 4;    // actions

// Offset of W^T[out][in] in a tiled [N][K] block (K = padded fan-in, N and K
// multiples of 16).
__host__ __device__ constexpr int qn_wt(int out, int in, int K) {
    return (((out >> 4) * (K >> 4) + (in >> 4)) << 8) + (((in >> 3) & 1) << 7) + ((out & 15) << 3) +
           (in & 7);
}

// Offset of W1^T[out][in] (in < 89) within the W1 block of an H-neuron layer.
template <int H>
__host__ __device__ constexpr int qn_w1(int out, int in) {
    return in < QN_DT ? (out >> 4) * (QN_DT * 16) + ((in >> 4) << 8) + (((in >> 3) & 1) << 7) +
                            ((out & 15) << 3) + (in & 7)
                      : QN_DT * H + out;
}

template <int H>
struct QL {
    static constexpr int oW1T = 0;
    static constexpr int oW1X = oW1T + H * QN_DT;  // feature 88's column W1T[:, 88]
    static constexpr int oW2T = oW1T + H * QN_D;
    static constexpr int oW3T = oW2T + H * H;
    static constexpr int ob1 = oW3T + QN_NA * H;
    static constexpr int ob2 = ob1 + H;
    static constexpr int ob3 = ob2 + H;
    static constexpr int P = ob3 + QN_NA;  // floats per agent (multiple of 4)
    static_assert(P % 4 == 0, "16-byte aligned agent rows");
    static_assert(oW2T % 8 == 0, "16-byte aligned f16 fragments of W2T");
};

}  // namespace dmdqn
