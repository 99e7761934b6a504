same as f_reconv; autoFit css-bobyqa retries in one launch per round
