def no_gpu():
    try:
        import torch
        return not torch.cuda.is_available()
    except Exception:
        return True
