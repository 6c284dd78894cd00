"""tossctr.configs restates the reference yamls the GPU box cannot read: pin the restatements to the
yamls themselves wherever /root/reference is present (the build container)."""
import os

import pytest

REF = "/root/reference/cfgs"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "dare_base.yaml")), reason="reference yamls absent")
def test_dare_base_equals_yaml():
    import yaml
    from tossctr.configs import dare_base
    with open(os.path.join(REF, "dare_base.yaml")) as f:
        ref = yaml.safe_load(f)
    assert dare_base() == ref


def test_dare_base_overrides_merge_sections():
    from tossctr.configs import dare_base
    cfg = dare_base(train={"batch_size": 256, "epochs": 1}, cv={"n_splits": 1})
    assert cfg["train"]["batch_size"] == 256 and cfg["train"]["lr"] == 0.001
    assert cfg["cv"] == {"n_splits": 1, "group_key": "inventory_id", "stratify_target": "clicked"}
