import sys, torch
a, b = torch.load(sys.argv[1]), torch.load(sys.argv[2])
for k in a:
    for i in range(2):
        print(k, i, "equal" if torch.equal(a[k][i], b[k][i]) else f"DIFF max {(a[k][i]-b[k][i]).abs().max().item():.3e}")
