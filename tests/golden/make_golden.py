"""Regenerates the committed golden fixtures of this directory from the C oracle (the CPU
restatement of the reference, oracle/).  Run from the repo root:  python tests/golden/make_golden.py

  squeezenet_synth_oracle.npz  synthetic SqueezeNet-1.0 (ore.squeezenet.build(224), seed 1234),
                               input = [zoo image squeezenet_data_0.pb, synthetic_input(1, seed 0)],
                               output = oracle softmax rows [2, 1000]
  squeezenet_synth8_oracle.npz the same model on 8 images: the zoo image + synthetic_input(7, seed 21)
                               (the benched plan's parity margin, tests/test_config4_gpu.py); also
                               squeezenet_synth8_f64.npz, the float64 executor's output (f64_ref.py)
  squeezenet_calib16_oracle.npz the zoo-calibrated model (ore.squeezenet.build_calibrated(): conv10 x
                               ZOO_LOGIT_GAIN, zoo-image softmax max 0.074 like squeezenet_output_0.pb)
                               on 16 images: the zoo image + synthetic_input(15, seed 31); the strict
                               1e-5 parity set of bench.py's plan (tests/test_config4_gpu.py) and
                               bench.py's max-abs sample; also squeezenet_calib16_f64.npz (f64_ref.py)
  squeezenet_mini_oracle.npz   the same topology at 64x64 input, 4 seeded images; also every
                               intermediate value of image 0 (for node-level parity)
  mnist_oracle.npz             mnist-8.onnx on mnist_data_0.pb and 3 derived images

The reference data files (mnist-8.onnx, *.pb) are copied verbatim from the reference repo's
fixtures; the .npz files are outputs of oracle/ (pinned against mnist_output_0.pb).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))

import oracle  # noqa: E402
from ore import onnx_wire, squeezenet  # noqa: E402


def squeezenet_inputs():
    zoo = onnx_wire.load_tensor(os.path.join(HERE, "squeezenet_data_0.pb")).to_numpy()
    return np.concatenate([zoo, squeezenet.synthetic_input(1, 224, seed=0)]).astype(np.float32)


def squeezenet_inputs8():
    zoo = onnx_wire.load_tensor(os.path.join(HERE, "squeezenet_data_0.pb")).to_numpy()
    return np.concatenate([zoo, squeezenet.synthetic_input(7, 224, seed=21)]).astype(np.float32)


def squeezenet_inputs_calib16():
    zoo = onnx_wire.load_tensor(os.path.join(HERE, "squeezenet_data_0.pb")).to_numpy()
    return np.concatenate([zoo, squeezenet.synthetic_input(15, 224, seed=31)]).astype(np.float32)


def mini_inputs():
    return squeezenet.synthetic_input(4, 64, seed=5)


def mnist_inputs():
    x = onnx_wire.load_tensor(os.path.join(HERE, "mnist_data_0.pb")).to_numpy()
    rng = np.random.default_rng(9)
    extra = rng.uniform(-30, 30, size=(3, 1, 28, 28)).astype(np.float32)
    return np.concatenate([x, extra]).astype(np.float32)


def synth8():
    import f64_ref
    model = squeezenet.build(224)
    x = squeezenet_inputs8()
    y = oracle.Model(model).run(x, 1000)
    np.savez_compressed(os.path.join(HERE, "squeezenet_synth8_oracle.npz"), output=y)
    y64 = np.concatenate([f64_ref.run(model, x[i:i + 1]) for i in range(x.shape[0])])
    np.savez_compressed(os.path.join(HERE, "squeezenet_synth8_f64.npz"), output=y64)


def calib16():
    import f64_ref
    model = squeezenet.build_calibrated(224)
    x = squeezenet_inputs_calib16()
    y = oracle.Model(model).run(x, 1000)
    np.savez_compressed(os.path.join(HERE, "squeezenet_calib16_oracle.npz"), output=y)
    y64 = np.concatenate([f64_ref.run(model, x[i:i + 1]) for i in range(x.shape[0])])
    np.savez_compressed(os.path.join(HERE, "squeezenet_calib16_f64.npz"), output=y64)


def main():
    if "--only-synth8" in sys.argv:
        synth8()
        print("wrote synth8 fixtures")
        return
    if "--only-calib16" in sys.argv:
        calib16()
        print("wrote calib16 fixtures")
        return
    synth8()
    calib16()
    m = oracle.Model(squeezenet.build(224))
    y = m.run(squeezenet_inputs(), 1000)
    np.savez_compressed(os.path.join(HERE, "squeezenet_synth_oracle.npz"), output=y)

    mini = squeezenet.build(64)
    m = oracle.Model(mini)
    x = mini_inputs()
    y = m.run(x, 1000)
    np.savez_compressed(os.path.join(HERE, "squeezenet_mini_oracle.npz"), output=y)

    with open(os.path.join(HERE, "mnist-8.onnx"), "rb") as f:
        m = oracle.Model(f.read())
    y = m.run(mnist_inputs(), 10)
    np.savez_compressed(os.path.join(HERE, "mnist_oracle.npz"), output=y)
    print("wrote fixtures")


if __name__ == "__main__":
    main()
