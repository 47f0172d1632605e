"""Drop-in for the reference's metrics.py (accuracy, micro/macro F1)."""


def accuracy(output, labels):
    """Fraction of argmax predictions equal to labels, as a 0-d double tensor
    (reference metrics.py:3-7)."""
    preds = output.max(1)[1].type_as(labels)
    return preds.eq(labels).double().sum() / len(labels)


def f1(output, labels):
    """(micro, macro) F1 via sklearn on host copies (reference metrics.py:9-15)."""
    from sklearn.metrics import f1_score
    preds = output.max(1)[1].cpu().detach().numpy()
    labels = labels.cpu().detach().numpy()
    return f1_score(labels, preds, average="micro"), f1_score(labels, preds, average="macro")
