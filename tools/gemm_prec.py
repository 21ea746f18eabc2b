import torch
torch.manual_seed(0)
for (m,k,n) in [(256,2304,960),(2304,256,960),(256,960,2304)]:
    a=torch.randn(m,k); b=torch.randn(k,n)
    ref=(a.double()@b.double())
    for name, fn in [('mm', lambda x,y: x@y)]:
        got=fn(a.cuda(), b.cuda()).double().cpu()
        print(m,k,n,name,'rel', float((got-ref).norm()/ref.norm()))
x=torch.randn(32,256,6,5,requires_grad=True); w=torch.randn(256,256,3,3,requires_grad=True)
for en in [False, True]:
    torch.backends.cudnn.enabled=en
    xd=x.detach().double().requires_grad_(); wd=w.detach().double().requires_grad_()
    y=torch.nn.functional.conv2d(xd,wd,padding=1); y.sum().backward()
    xc=x.detach().cuda().requires_grad_(); wc=w.detach().cuda().requires_grad_()
    yc=torch.nn.functional.conv2d(xc,wc,padding=1); yc.sum().backward()
    print('cudnn',en,'fwd',float((yc.double().cpu()-y).norm()/y.norm()),'dx',float((xc.grad.double().cpu()-xd.grad).norm()/xd.grad.norm()),'dw',float((wc.grad.double().cpu()-wd.grad).norm()/wd.grad.norm()))
# train-mode BatchNorm2d forward/backward vs float64
for en in [False, True, False]:
    torch.backends.cudnn.enabled = en
    torch.manual_seed(1)
    x = torch.randn(32, 256, 6, 5) * 3 + 1
    r = torch.randn(32, 256, 6, 5)
    bd = torch.nn.BatchNorm2d(256).double().train()
    xd = x.double().requires_grad_()
    (bd(xd) * r.double()).sum().backward()
    bc = torch.nn.BatchNorm2d(256).cuda().train()
    xc = x.cuda().requires_grad_()
    (bc(xc) * r.cuda()).sum().backward()
    rel = lambda a, b: float((a.double().cpu() - b).norm() / b.norm())
    print('bn cudnn', en, 'dx', rel(xc.grad, xd.grad), 'dgamma', rel(bc.weight.grad, bd.weight.grad), 'dbeta',
          rel(bc.bias.grad, bd.bias.grad), 'running_var', rel(bc.running_var, bd.running_var))
