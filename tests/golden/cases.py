"""Configurations of the reference-generated ``predict_*.npz`` fixtures (tests/golden/make_golden.py writes them,
tests/test_gpu_predict_modes.py replays them): name -> (SPEUtils positional args after ``camera``, URSONet head
widths (n_ori, n_pos), ``synthetic_state_dict`` keyword args, frames (b, h, w, seed))."""

PREDICT_CASES = {
    # SPEUtils default histogram (ORI_DELETE_UNUSED_BINS=True -> 1232 bins), position regression at SPEED range
    'predict_cls1232_posreg': (('classification', 12, 3, True, 'regression'), (1232, 3),
                               dict(head_std=0.3, pos_std=0.01, pos_bias=(0.3, -0.2, 12.0)), (3, 160, 224, 21)),
    # 1728-bin orientation + 1000-bin position soft classification (POS: classification)
    'predict_cls1728_poscls': (('classification', 12, 3, False, 'classification'), (1728, 1000),
                               dict(head_std=0.3, pos_std=0.05), (3, 128, 192, 22)),
    # orientation regression (L2 normalise, spe_utils.py:72) + position regression
    'predict_orireg_posreg': (('regression', 12, 3, True, 'regression'), (4, 3),
                              dict(head_std=0.01, pos_bias=(-1.1, 0.7, 25.0)), (3, 160, 224, 23)),
}
