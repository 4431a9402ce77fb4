"""dmdqn_amd -- MI355X-native hot path of pranshu-raj-211/dmdqn.

The vectorised traffic microsimulation (replacing SUMO/TraCI), observation and
reward assembly, epsilon-greedy act, replay store/sample and the Double-DQN
learn step run as hand-written gfx950 HIP kernels behind a C ABI
(include/dmdqn.h, built into dmdqn_amd/lib/libdmdqn_hip.so).  Python mirrors
the reference's Env / DQNAgent surfaces on top.
"""
__version__ = "0.1.0"
