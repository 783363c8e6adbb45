"""MNIST CNN (reference hetseq/tasks/tasks.py:318-343, eval variant eval_mnist.py:19-36).

conv(1->32,3) -> ReLU -> conv(32->64,3) -> ReLU -> maxpool2 -> dropout2d(0.25) ->
fc 9216->128 -> ReLU -> dropout2d(0.5) -> fc 128->10 -> log_softmax -> NLL.
A plumbing task: convolutions go to MIOpen through torch on the GPU.
Note: the reference applies ``Dropout2d`` to a 2-D [N, 128] activation, which
torch treats as channel dropout over the batch dim; ``F.dropout2d`` on 2-D input
is kept for behavioural parity.
"""
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F


class MNISTNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout2d(0.25)
        self.dropout2 = nn.Dropout2d(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x, target=None, eval=False):
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            x = self.dropout2(x)
        x = self.fc2(x)
        output = F.log_softmax(x, dim=1)
        if target is None:
            return output
        loss = F.nll_loss(output, target)
        if eval:
            return output, loss
        return loss
