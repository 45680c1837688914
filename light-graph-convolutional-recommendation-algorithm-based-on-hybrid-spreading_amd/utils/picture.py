"""Line plot helper with the reference's signature (reference utils/picture.py:11), imported
by the training loops' curve output and by findLambda.py. Off the hot path: plain matplotlib
(Agg backend, so it works on a headless GPU box); the directory of ``save_path`` is created
on demand, like every other writer of this package."""
import os


def plotMetric(xpoints: list, ypoints: list, xlabel: str, ylabel: str, title: str,
               save_path: str) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    d = os.path.dirname(save_path)
    if d:
        os.makedirs(d, exist_ok=True)
    fig = plt.figure()
    plt.plot(xpoints, ypoints)
    plt.xlabel(xlabel)
    plt.ylabel(ylabel)
    plt.title(title)
    plt.savefig(save_path)
    plt.close(fig)
