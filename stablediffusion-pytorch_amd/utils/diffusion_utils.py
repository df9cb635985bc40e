"""Classifier-free-guidance condition dropping (API mirror of reference utils/diffusion_utils.py:21-46).

Device RNG draws the per-sample keep/drop decision exactly as the reference does (uniform_ on a
(B,...) float tensor on the input's device)."""
import torch


def drop_text_condition(text_embed, im, empty_text_embed, text_drop_prob):
    if text_drop_prob > 0:
        drop = torch.zeros((im.shape[0]), device=im.device).float().uniform_(0, 1) < text_drop_prob
        assert empty_text_embed is not None, ("Text Conditioning required as well as"
                                              " text dropping but empty text representation not created")
        text_embed[drop, :, :] = empty_text_embed[0]
    return text_embed


def drop_image_condition(image_condition, im, im_drop_prob):
    if im_drop_prob > 0:
        keep = torch.zeros((im.shape[0], 1, 1, 1), device=im.device).float().uniform_(0, 1) > im_drop_prob
        return image_condition * keep
    return image_condition


def drop_class_condition(class_condition, class_drop_prob, im):
    if class_drop_prob > 0:
        keep = torch.zeros((im.shape[0], 1), device=im.device).float().uniform_(0, 1) > class_drop_prob
        return class_condition * keep
    return class_condition
