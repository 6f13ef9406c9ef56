"""PyTorch definitions of the networks the ONNX / PyTorch examples export
(reference examples/python/onnx/*_pt.py and examples/python/pytorch/*_torch.py)."""
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1, self.linear2, self.linear3 = nn.Linear(784, 512), nn.Linear(512, 512), nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        return self.softmax(self.linear3(self.relu(self.linear2(self.relu(self.linear1(x))))))


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1, self.conv2 = nn.Conv2d(3, 32, 3, 1, 1), nn.Conv2d(32, 32, 3, 1, 1)
        self.conv3, self.conv4 = nn.Conv2d(32, 64, 3, 1, 1), nn.Conv2d(64, 64, 3, 1, 1)
        self.pool1, self.pool2 = nn.MaxPool2d(2, 2), nn.MaxPool2d(2, 2)
        self.flat = nn.Flatten()
        self.linear1, self.linear2 = nn.Linear(64 * 8 * 8, 512), nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        r = self.relu
        x = self.pool1(r(self.conv2(r(self.conv1(x)))))
        x = self.pool2(r(self.conv4(r(self.conv3(x)))))
        return self.softmax(self.linear2(r(self.linear1(self.flat(x)))))


class AlexNet(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 11, 4, 2), nn.ReLU(), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, 1, 2), nn.ReLU(), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, 1, 1), nn.ReLU(), nn.Conv2d(384, 256, 3, 1, 1), nn.ReLU(),
            nn.Conv2d(256, 256, 3, 1, 1), nn.ReLU(), nn.MaxPool2d(3, 2))
        self.flat = nn.Flatten()
        self.classifier = nn.Sequential(nn.Linear(256 * 6 * 6, 4096), nn.ReLU(), nn.Linear(4096, 4096), nn.ReLU(),
                                        nn.Linear(4096, num_classes), nn.Softmax(dim=1))

    def forward(self, x):
        return self.classifier(self.flat(self.features(x)))


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU()
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, 0, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = self.bn2(self.conv2(self.relu(self.bn1(self.conv1(x)))))
        return self.relu(y + (self.down(x) if self.down is not None else x))


class ResNet(nn.Module):
    """ResNet-18-style network for 3x32x32 inputs (reference onnx/resnet_pt.py exports a torchvision-
    style ResNet; sized here for CIFAR-10)."""

    def __init__(self, num_classes=10, widths=(64, 128, 256, 512)):
        super().__init__()
        self.conv1 = nn.Conv2d(3, widths[0], 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(widths[0])
        self.relu = nn.ReLU()
        blocks, cin = [], widths[0]
        for i, w in enumerate(widths):
            blocks += [BasicBlock(cin, w, 1 if i == 0 else 2), BasicBlock(w, w)]
            cin = w
        self.layers = nn.Sequential(*blocks)
        self.pool = nn.AvgPool2d(4, 4)
        self.flat = nn.Flatten()
        self.fc = nn.Linear(widths[-1], num_classes)
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        x = self.layers(self.relu(self.bn1(self.conv1(x))))
        return self.softmax(self.fc(self.flat(self.pool(x))))
