"""Dump the reference's own model configs as a JSON fixture (runs in the build container only).

    python tests/golden/make_hparams_golden.py

Imports the reference's pure-Python config modules
    /root/reference/automl/efficientdet/hparams_config.py      (get_efficientdet_config, :301-480)
    /root/reference/automl/efficientdet/tf2/fpn_configs.py     (get_fpn_config, :166-176)
with a stub `tensorflow` module in sys.modules: both only use TF for YAML file I/O
(tf.io.gfile), which is never called here.  The output, tests/golden/hparams_configs.json, is data
(config values and BiFPN node lists per model); tests/test_kats.py checks the product's model table
(libphx phx_model_info) and the oracle's table against it.  /root/reference does not exist on the
GPU box; only the JSON travels.
"""
import json
import os
import sys
import types

REF = "/root/reference/automl/efficientdet"
HERE = os.path.dirname(os.path.abspath(__file__))

MODELS = [f"efficientdet-d{i}" for i in range(8)] + [f"efficientdet-lite{i}" for i in range(5)]
KEYS = ["name", "backbone_name", "image_size", "fpn_num_filters", "fpn_cell_repeats", "box_class_repeats",
        "anchor_scale", "num_scales", "aspect_ratios", "min_level", "max_level", "act_type", "fpn_weight_method",
        "fpn_name", "mean_rgb", "stddev_rgb", "num_classes", "nms_configs", "apply_bn_for_resampling",
        "conv_after_downsample", "separable_conv", "conv_bn_act_pattern", "survival_prob", "is_training_bn"]


def main():
    stub = types.ModuleType("tensorflow")
    stub.io = types.SimpleNamespace(gfile=types.SimpleNamespace(GFile=None))
    sys.modules.setdefault("tensorflow", stub)
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "tf2"))
    import hparams_config  # noqa: E402  (reference module)
    import fpn_configs  # noqa: E402  (reference module)

    out = {}
    for m in MODELS:
        c = hparams_config.get_efficientdet_config(m).as_dict()
        d = {k: c.get(k) for k in KEYS}
        fpn = fpn_configs.get_fpn_config(c.get("fpn_name"), c["min_level"], c["max_level"],
                                         c.get("fpn_weight_method"))
        d["fpn_effective_weight_method"] = fpn.weight_method
        d["fpn_nodes"] = [{"feat_level": n["feat_level"], "inputs_offsets": list(n["inputs_offsets"])}
                          for n in fpn.nodes]
        out[m] = d
    # attacker_train.py:31 override on top of the default nms_configs (Config.override, :91-109)
    c = hparams_config.get_efficientdet_config("efficientdet-lite4")
    c.override({"nms_configs": {"iou_thresh": .5, "score_thresh": .5}})
    out["_attacker_train_override"] = {"nms_configs": c.as_dict()["nms_configs"]}
    path = os.path.join(HERE, "hparams_configs.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(path)


if __name__ == "__main__":
    main()
