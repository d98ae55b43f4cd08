"""Global confidence threshold: ``Licensee.confidence_threshold`` (lib/licensee.rb:21,47-54)."""

CONFIDENCE_THRESHOLD = 98
_threshold = None


def confidence_threshold():
    return CONFIDENCE_THRESHOLD if _threshold is None else _threshold


def set_confidence_threshold(value):
    global _threshold
    _threshold = value
