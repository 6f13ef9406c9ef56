"""ResNet-50 (examples/cpp/ResNet/resnet.cc; python/native/resnet.py) on random data: the reference apps' synthetic mode
(one random batch loaded once, timed forward / zero_gradients / backward / update loop).

    python examples/python/native/resnet.py -b 64 -e 1 [--iterations N] [--small]
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import fill_synthetic, header, report  # noqa: E402

from flexmi.core import FFConfig, FFModel, SGDOptimizer  # noqa: E402
from flexmi.models import zoo  # noqa: E402


def main():
    cfg = FFConfig()
    cfg.parse_args()
    small = "--small" in sys.argv
    header(cfg)
    model = FFModel(cfg)
    built = zoo.build("resnet50", model, small=small)
    model.compile(SGDOptimizer(model, built.lr), built.loss, built.metrics)
    model.init_layers()
    fill_synthetic(model, list(built.inputs.values()), classes=built.output.dims[-1])
    iters = max(1, cfg.iterations)
    model.forward(); model.zero_gradients(); model.backward(); model.update()   # warm-up
    t0 = cfg.get_current_time()
    for _ in range(cfg.get_epochs()):
        for _ in range(iters):
            model.forward()
            model.zero_gradients()
            model.backward()
            model.update()
    report(cfg, cfg.get_batch_size() * iters, cfg.get_epochs(), t0, cfg.get_current_time())


if __name__ == "__main__":
    print("resnet50")
    main()
