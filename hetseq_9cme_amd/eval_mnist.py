"""Post-hoc MNIST test-set evaluation of a checkpoint (reference hetseq/eval_mnist.py:39-100).

``python -m hetseq_9cme_amd.eval_mnist --mnist_dir DATA --model_ckpt CKPT``
prints average loss and accuracy on the test split (reads checkpoint['model']).
"""
import argparse

import torch
import torch.nn.functional as F

from .checkpoint_utils import load_checkpoint_to_cpu
from .data.mnist_dataset import MNISTDataset
from .models.mnist import MNISTNet


def evaluate(model_ckpt, mnist_dir, device=None, batch_size=64, verbose=False):
    device = torch.device(device or ('cuda' if torch.cuda.is_available() else 'cpu'))
    state = load_checkpoint_to_cpu(model_ckpt)
    model = MNISTNet()
    model.load_state_dict(state['model'])
    model.to(device).eval()
    ds = MNISTDataset.from_path(mnist_dir, 'test')
    test_loss, correct = 0.0, 0
    with torch.no_grad():
        for i in range(0, len(ds), batch_size):
            x = ds.image[i:i + batch_size].to(device)
            y = ds.label[i:i + batch_size].to(device)
            out, loss = model(x, y, eval=True)
            test_loss += F.nll_loss(out, y, reduction='sum').item()
            correct += (out.argmax(dim=1) == y).sum().item()
    n = len(ds)
    if verbose:
        print('\nTest set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n'.format(
            test_loss / n, correct, n, 100. * correct / n))
    return correct / n


def main(argv=None):
    p = argparse.ArgumentParser(description='evaluate trained mnist model')
    p.add_argument('--mnist_dir', type=str, required=True)
    p.add_argument('--model_ckpt', type=str, required=True)
    p.add_argument('--cpu', action='store_true')
    a = p.parse_args(argv)
    evaluate(a.model_ckpt, a.mnist_dir, device='cpu' if a.cpu else None, verbose=True)


if __name__ == '__main__':
    main()
