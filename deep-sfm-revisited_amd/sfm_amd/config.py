"""Hot-path subset of the reference's global config (lib/config.py + cfgs/kitti.yml).

Only the flags the RANSAC-pose and plane-sweep path reads are kept; defaults
follow lib/config.py, and ``kitti()`` applies cfgs/kitti.yml's overrides.
"""


class Config(dict):
    """Attribute-access dict (the reference uses easydict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def defaults():
    return Config(
        ransac_iter=5,            # lib/config.py:53
        ransac_threshold=1e-4,    # lib/config.py:54
        min_matches=20,           # lib/config.py:55
        MIN_DEPTH=1.0,            # lib/config.py:26
        NORM_TARGET=0.8,          # lib/config.py:40
        RESCALE_DEPTH=False,      # lib/config.py:130
        MIXED_PREC=False,         # lib/config.py:172
        PRED_POSE_ONLINE=True,    # lib/config.py:42
        POSE_EST="RANSAC",        # lib/config.py:51
        GT_POSE=False,            # lib/config.py:198
        GT_POSE_NORMALIZED=False, # lib/config.py:200
        PRED_POSE_GT_SCALE=False, # lib/config.py:144
        RECORD_POSE=False,        # lib/config.py:147
        RECORD_POSE_EVAL=False,   # lib/config.py:149
        PREDICT_BY_DEPTH=False,   # lib/config.py:91
        TRAIN_FLOW=False,         # lib/config.py
        FLOW_EST="DICL",          # lib/config.py:178 (RAFT / DICL: out of scope, injected)
        DEPTH_EST="PSNET",        # lib/config.py:181 (PSNET built by default; others injected)
        PSNET_CONTEXT=True,       # lib/config.py:46
        PSNET_DEP_CONTEXT=False,  # lib/config.py:47
        IND_CONTEXT=False,        # lib/config.py:164
        CONTEXT_BN=False,         # lib/config.py:158
    )


def kitti():
    c = defaults()
    c.update(MIXED_PREC=True, RESCALE_DEPTH=True, NORM_TARGET=0.6, MIN_DEPTH=1.0, ransac_iter=5,
             PRED_POSE_ONLINE=True, PSNET_DEP_CONTEXT=True)   # cfgs/kitti.yml:10-41
    return c


cfg = defaults()
